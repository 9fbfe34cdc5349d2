"""Make the sibling ``mhada_hip`` runtime importable when only this package's parent
directory is on sys.path (the drop-in usage: ``sys.path.insert(0, ".../mhada-style-transfer_amd")``)."""
import os
import sys

_PARENT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PARENT not in sys.path:
    sys.path.insert(0, _PARENT)

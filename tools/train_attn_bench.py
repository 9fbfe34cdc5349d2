"""Time the training attention kernels at the train_image.py 512^2 B8 block shape
(BH = 64, Nc = Ns = 4096): forward, backward (dQ + dK/dV'), per-kernel averages via HIP events.
usage: python tools/train_attn_bench.py [reps]"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "mhada-style-transfer_amd")]
import torch  # noqa: E402

from mhada_hip import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
libs = sys.argv[2:]  # optional: A/B of several builds in this process (interleaved, median of 5)
BH, N = 64, 4096
g = torch.Generator(device="cuda").manual_seed(0)
q, k, x = (torch.randn(BH, N, 64, device="cuda", generator=g) * 0.3 for _ in range(3))
v = torch.randn(BH, N, 64, device="cuda", generator=g)
out, mo, lse = ops.attn_train_fwd(q, k, v, x)
dmo = torch.randn(BH, N, 128, device="cuda", generator=g)
dd = torch.randn(BH, N, device="cuda", generator=g)
pairs = BH * N * N


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


if libs:
    from mhada_hip import _lib
    handles = {p: _lib.load(p) for p in libs}
    res = {p: [] for p in libs}
    for _ in range(5):
        for p in libs:
            _lib._lib = handles[p]
            res[p].append((timeit(lambda: ops.attn_train_fwd(q, k, v, x)),
                           timeit(lambda: ops.attn_train_bwd(q, k, v, lse, dmo, dd, spill=False)),
                           timeit(lambda: ops.attn_train_bwd(q, k, v, lse, dmo, dd, spill=True))))
    for p in libs:
        med = [sorted(r[i] for r in res[p])[2] for i in range(3)]
        print(f"{p}: fwd {med[0]:.3f} ms  bwd recompute {med[1]:.3f} ms  bwd dS spill {med[2]:.3f} ms")
    sys.exit(0)
tf = timeit(lambda: ops.attn_train_fwd(q, k, v, x))
tb = timeit(lambda: ops.attn_train_bwd(q, k, v, lse, dmo, dd, spill=False))
ts = timeit(lambda: ops.attn_train_bwd(q, k, v, lse, dmo, dd, spill=True))
print(f"fwd {tf:.3f} ms ({384 * pairs / tf / 1e9:.1f} TF)  "
      f"bwd recompute {tb:.3f} ms ({1280 * pairs / tb / 1e9:.1f} TF)  "
      f"bwd dS spill {ts:.3f} ms ({896 * pairs / ts / 1e9:.1f} TF of the 896-FLOP form)")

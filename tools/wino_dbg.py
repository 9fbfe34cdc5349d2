"""Ablation timing of the Winograd conv kernel: builds of wino.hip with -DWINO_DBG=<bits> (1 no
MFMA, 2 no global loads, 4 no transform / LDS stores) linked as build_dbg/libwino_<bits>.so,
timed on one shape, for each value of the tuning knob WINO_KNOB (default xknob: 0 and 1).
usage: python tools/wino_dbg.py B H Ci Co [bits ...]   (WINO_LIB_DIR: directory of the builds)"""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import torch

B, H, Ci, Co = map(int, sys.argv[1:5])
bits = [int(v) for v in sys.argv[5:]] or [0, 1, 2, 4, 6, 7]
x = torch.rand(B, H, H, Ci, device="cuda")
w = torch.randn(Co, 9 * Ci, device="cuda") / (9 * Ci) ** 0.5
u = torch.empty(Ci // 8, 16, Co, 8, device="cuda")
y = torch.empty(B, H, H, Co, device="cuda")
st = torch.cuda.current_stream().cuda_stream
flop = 2.0 * 9 * Ci * Co * B * H * H
for v in bits:
    lib = ctypes.CDLL(os.path.join(REPO, "mhada-style-transfer_amd", os.environ.get("WINO_LIB_DIR", "build_dbg"), f"libwino_{v}.so"))
    lib.mhada_conv3x3_wino.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 5 + [ctypes.c_longlong] + \
        [ctypes.c_int] * 3 + [ctypes.c_void_p] * 2
    lib.mhada_set_tuning.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lib.mhada_wino_weights.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    assert lib.mhada_wino_weights(w.data_ptr(), u.data_ptr(), Co, Ci, st) == 0
    f = lambda: lib.mhada_conv3x3_wino(x.data_ptr(), u.data_ptr(), None, y.data_ptr(), B, H, H, Ci, Co, Co, 0, 1, 1, None, st)  # noqa
    for kv in [int(v) for v in os.environ.get("WINO_KNOB_VALS", "0,1").split(",")]:
        assert lib.mhada_set_tuning(os.environ.get("WINO_KNOB", "xknob").encode(), kv) == 0
        f(); torch.cuda.synchronize()
        ts = []
        for _ in range(15):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(); f(); e.record(); torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) * 1e3)
        t = sorted(ts)[len(ts) // 2]
        print(f"WINO_DBG={v} knob={kv}: {t:8.1f} us  ({flop / 2.25 / t / 1e6:6.1f} TF/s MFMA-equiv)", flush=True)

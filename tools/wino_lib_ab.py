"""Interleaved A/B of two wino.hip builds (build_ab/libwino_<a>.so vs libwino_<b>.so, built with
different -D flags): alternating rounds on the same operands, median per build and shape.
usage: WINO_LIB_DIR=build_ab python tools/wino_lib_ab.py a b [rounds]"""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import torch

a, b = sys.argv[1], sys.argv[2]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 9
d = os.path.join(REPO, "mhada-style-transfer_amd", os.environ.get("WINO_LIB_DIR", "build_ab"))
libs = {}
for v in (a, b):
    lib = ctypes.CDLL(os.path.join(d, f"libwino_{v}.so"))
    lib.mhada_conv3x3_wino.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 5 + [ctypes.c_longlong] + \
        [ctypes.c_int] * 3 + [ctypes.c_void_p]
    lib.mhada_wino_weights.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    libs[v] = lib
st = torch.cuda.current_stream().cuda_stream
for (B, H, Ci, Co, pm) in [(8, 128, 256, 256, 0), (8, 512, 64, 64, 0), (8, 256, 128, 128, 0), (8, 64, 512, 256, 0),
                           (8, 512, 64, 64, 1), (8, 128, 256, 256, 1)]:
    x = torch.rand(B, H, H, Ci, device="cuda")
    w = torch.randn(Co, 9 * Ci, device="cuda") / (9 * Ci) ** 0.5
    u = torch.empty(Ci // 8, 16, Co, 8, device="cuda")
    ys = {v: torch.empty(B, H, H, Co, device="cuda") for v in libs}
    ts = {v: [] for v in libs}
    for v, lib in libs.items():
        assert lib.mhada_wino_weights(w.data_ptr(), u.data_ptr(), Co, Ci, st) == 0
    for r in range(rounds + 1):
        for v, lib in libs.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                lib.mhada_conv3x3_wino(x.data_ptr(), u.data_ptr(), None, ys[v].data_ptr(), B, H, H, Ci, Co, Co, pm, 1, 1, None, st)
            e.record()
            torch.cuda.synchronize()
            if r:
                ts[v].append(s.elapsed_time(e) / 5 * 1e3)
    same = torch.equal(ys[a], ys[b])
    med = {v: sorted(t)[len(t) // 2] for v, t in ts.items()}
    print(f"B{B} {H}^2 {Ci}->{Co} pad{'zero' if pm else 'refl'}: " + "  ".join(f"{v} {m:8.1f} us" for v, m in med.items())
          + f"  ({med[b] / med[a]:.3f}x)  outputs equal: {same}", flush=True)

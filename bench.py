"""Benchmark: stylized frames/s of the MHAdaSTr forward path on MI355X (BASELINE.json).

A "step" is one full style-transfer forward — vit_c(content), vit_s(style),
adaFormer(fc, fs) (infer_image.py:83-85 / infer_time.py:74-77) — over one synthetic batch
already resident in HBM.  Headline workload = BASELINE configs[1]: 512x512, batch 8, fp32.
The line also carries configs[2] (1024x1024, batch 4, bf16 MFMA path), configs[3] (the
train_image.py step at 512x512, 8 images per GPU), configs[4] (1080p u8 video frames ingested,
stylised against a cached 256^2 style + warping error, fp32 and bf16) and the reference's own
latency probe (infer_time.py: B=1 512^2, eager and hipGraph-replayed) under "configs".

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

--gpus N > 1 without a launcher (WORLD_SIZE unset): bench.py starts the N rank processes itself
(one child per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, 127.0.0.1 rendezvous) BEFORE
this process makes any GPU call, relays their output and exits non-zero if any rank fails.
Under a launcher WORLD_SIZE must equal --gpus.

Multi-GPU: inference replicas: the ViT's batch-axis attention couples the
images of one forward call, so a call's batch is never split; each rank runs its own batch,
no collective on the data path (barrier + max-over-ranks timing only) -> scaling "weak".

Roofline: the dominant kernel is the fused MHAda attention (6 launches/step); its algorithmic FLOPs
per launch = 6*Nc*Ns*C*B (QK^T, PV, PV^2; 2 FLOP/MAC), timed live with HIP events on its launch
stream over the timed region.  The fp32 headline's attention (mhada_attn_split3) runs fp32-accurate
SPLIT3 products on the bf16 MFMA, so its line prices the bf16 MFMA FLOPs it issues (6.25x the
algorithmic fp32 FLOPs) against the bf16 peak and states the fp32-equivalent rate beside them.  After every timed region the same process
runs a shader-clock probe (csrc/probe.hip) and reports the box's clock under dense MFMA load
("clock_ghz"; "frac_at_clock" = the fraction of the peak scaled to that clock).  CPU baseline (rank 0, N=1): the
reference's aten fp32 expression (tests/torch_ref.py, golden-pinned) at B=1 on the job's host
cores, with the numpy oracle beside it.
"""
import argparse
import contextlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "mhada-style-transfer_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch
import torch.distributed as dist

PEAK_TFLOPS = {"f32": 157.3, "bf16": 2500.0}  # MI355X_MICROARCH.md: dense MFMA peaks
C = 512


class _mark:
    """A roctx range around a timed region ("bench:<config>:<steps>"): under `rocprofv3
    --marker-trace --kernel-trace` tools/ktrace.py assigns each kernel to the config whose timed
    region contains it (no profiler attached: a no-op)."""

    def __init__(self, name: str, steps: int):
        self.label = f"bench:{name}:{steps}"

    def __enter__(self):
        torch.cuda.nvtx.range_push(self.label)

    def __exit__(self, *exc):
        torch.cuda.nvtx.range_pop()
        return False


def max_over_ranks(x: float, world: int) -> float:
    """The job's time: max over ranks (RCCL on the GPU; gloo when MHADA_BENCH_BACKEND=gloo)."""
    if world == 1:
        return x
    dev = bench_device() if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def flops_per_frame(res: int, style_res: int) -> dict:
    """SURVEY.md §8(d) algorithmic FLOPs (2 FLOP/MAC)."""
    nc, ns = (res // 8) ** 2, (style_res // 8) ** 2
    d = 64
    vit = lambda n: 72 * n * C * C + 196608 * n  # noqa: E731  (+12*N*B*C batch-attn, negligible)
    mhada = 6 * (6 * nc * ns * C + 2 * (nc + 2 * ns) * C * d + 2 * nc * C * C)
    dec = 30892032 * nc
    return {"total": vit(nc) + vit(ns) + mhada + dec, "attn_per_block": 6 * nc * ns * C}


ATTN_SOURCES = ("mhada-style-transfer_amd/csrc/attn.hip", "mhada-style-transfer_amd/csrc/attn_split3.hip",
                "mhada-style-transfer_amd/csrc/attn_common.h", "mhada-style-transfer_amd/csrc/common.h")

# The fp32 softmax attention runs as SPLIT3 products on the bf16 MFMA (csrc/attn_split3.hip, round 6):
# per (query, key, head) 6 x 128 (Q K^T) + 6 x 256 (P [V' | V'^2]) + 3 x 32 (row sum, all-ones A)
# bf16 MFMA FLOP for the 384 algorithmic fp32 FLOP
SPLIT3_MFMA_PER_FP32 = (6 * 128 + 6 * 256 + 3 * 32) / 384


def attn_source_sha() -> str:
    """sha256 (16 hex) of the attention kernel's sources: ties a PMC measurement to this build.
    Comments and blank lines are left out (round 6), so a comment edit keeps a measurement valid;
    any change to the code itself makes it stale."""
    import hashlib
    import re
    h = hashlib.sha256()
    for rel in ATTN_SOURCES:
        with open(os.path.join(REPO, rel), encoding="utf-8") as f:
            text = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
        for line in text.splitlines():
            line = line.split("//", 1)[0].rstrip()
            if line:
                h.update(line.encode() + b"\n")
    return h.hexdigest()[:16]


def pmc_traffic(cfg_key):
    """HBM bytes per mhada_attn launch from the latest committed rocprofv3 PMC pass
    (profiles/rNN_pmc_traffic.json, produced by tools/pmc_traffic.py; FETCH_SIZE x2 + WRITE_SIZE
    per the gfx950 corrections).  PMC counters need their own profiler run, so the bench reads
    the measured value rather than collecting it live — and only when that pass measured THIS
    attention kernel source (attn_src_sha recorded by tools/pmc_traffic.py); otherwise null."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_traffic.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        doc = json.load(f)
    d = doc.get(cfg_key)
    if not d or doc.get("attn_src_sha") != attn_source_sha():
        return None, f"{os.path.relpath(files[-1], REPO)} (stale: other attention source)" if d else None
    return d["traffic_bytes_per_launch"], os.path.relpath(files[-1], REPO)


def shader_clock(launches: int = 20, iters: int = 150000) -> float:
    """The box's sustained shader clock under dense bf16 MFMA load, in GHz, measured in THIS process
    right after a timed region (mhada_clock_probe, csrc/probe.hip: s_memtime / s_memrealtime around a
    dependent MFMA chain per workgroup, ~10 ms per launch, `launches` back to back; median over the
    workgroups of the last launch).  The chip's clock under load differs between boxes by up to
    ~10 % (MI355X_MICROARCH.md, DVFS give-back), so this number separates a code change from a box
    change between two bench lines."""
    from mhada_hip import _lib
    lib = _lib.load()
    dev = bench_device()
    n = torch.cuda.get_device_properties(dev).multi_processor_count
    buf = torch.zeros(2 * n, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(launches):
        _lib.check(lib.mhada_clock_probe(buf.data_ptr(), n, iters, st), "mhada_clock_probe")
    torch.cuda.synchronize(dev)
    v = buf.view(n, 2).double().cpu()
    ghz = (v[:, 0] / v[:, 1].clamp(min=1) * 0.1).sort().values
    return round(float(ghz[n // 2]), 4)


PEAK_CLOCK_GHZ = 2.4  # the clock the dense peaks above are quoted at (MI355X_MICROARCH.md)


def build_models(dtype):
    import network
    from mhada_hip.recipe import load_recipe
    dev = torch.device("cuda", torch.cuda.current_device())
    vc = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c").to(dev).eval()
    vs = load_recipe(network.VisionTransformer(pos_embedding=False), "vit_s").to(dev).eval()
    ada = load_recipe(network.AdaAttnTransformerMultiHead(), "ada").to(dev).eval()
    for m in (vc, vs, ada):
        m.compute_dtype = dtype
    return vc, vs, ada


def run_config(res, batch, dtype, steps, warmup, rank, world):
    from mhada_hip import engine
    from mhada_hip.recipe import seeded_image
    vc, vs, ada = build_models(dtype)
    dev = torch.device("cuda", torch.cuda.current_device())
    c = seeded_image(batch, res, res, 11 + 1000 * rank).to(dev)
    s = seeded_image(batch, res, res, 12 + 1000 * rank).to(dev)

    def step():
        fc = vc(c)
        fs = vs(s)
        return ada(fc, fs)

    with torch.no_grad():
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        log = {}
        engine.record_kernel_events(log)
        t0 = time.perf_counter()
        with _mark(f"{res}x{res}_b{batch}_{'f32' if dtype == torch.float32 else 'bf16'}", steps):
            for _ in range(steps):
                out = step()
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        engine.record_kernel_events(None)
    assert torch.isfinite(out[1]).all()
    clock = shader_clock()
    ev = log.get("mhada_attn", [])
    attn_ms = [a.elapsed_time(b) for a, b in ev]
    elapsed = max_over_ranks(elapsed, world)
    frames = batch * steps * world
    dts = "f32" if dtype == torch.float32 else "bf16"
    fl = flops_per_frame(res, res)
    avg_attn_s = (sum(attn_ms) / len(attn_ms)) / 1e3 if attn_ms else float("nan")
    attn_flops = fl["attn_per_block"] * batch
    traffic, tsrc = pmc_traffic(f"{res}x{res}_b{batch}_{dts}")
    from mhada_hip import ops
    split3 = dtype == torch.float32 and ops.F32_SPLIT_ATTN
    if split3:
        # priced against the pipe it runs on: bf16 MFMA FLOP / 2.5 PF; the fp32-equivalent rate
        # (algorithmic fp32 FLOP / time, against the fp32 MFMA peak) is stated beside it
        mfma_flops = attn_flops * SPLIT3_MFMA_PER_FP32
        achieved, peak = mfma_flops / avg_attn_s / 1e12, PEAK_TFLOPS["bf16"]
    else:
        mfma_flops = attn_flops
        achieved, peak = attn_flops / avg_attn_s / 1e12, PEAK_TFLOPS[dts]
    roof = {"bound": "mfma", "kernel": "mhada_attn_split3" if split3 else "mhada_attn", "achieved": round(achieved, 2),
            "peak": peak, "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
            "traffic": traffic, "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": tsrc,
            "avg_launch_ms": round(avg_attn_s * 1e3, 4),
            "flop_per_launch": mfma_flops, "launches_timed": len(attn_ms),
            "clock_ghz": clock, "frac_at_clock": round(achieved / (peak * clock / PEAK_CLOCK_GHZ), 4)}
    if split3:
        roof["pipe"] = "bf16 MFMA (fp32-accurate SPLIT3 products: 3 bf16 planes per fp32 operand, 6 cross products)"
        roof["algorithmic_fp32_flop_per_launch"] = attn_flops
        roof["fp32_equiv_tflops"] = round(attn_flops / avg_attn_s / 1e12, 2)
        roof["fp32_equiv_frac_of_fp32_peak"] = round(attn_flops / avg_attn_s / 1e12 / PEAK_TFLOPS["f32"], 4)
    return {
        "value": frames / elapsed,
        "ms_per_step": elapsed / steps * 1e3,
        "dtype": dts,
        "frames_per_s_per_gpu": frames / elapsed / world,
        "tflops_whole_step": fl["total"] * batch * steps / (elapsed) / 1e12,
        "roofline": roof,
        "clock_ghz": clock,
        "config": {"workload": f"stylize {res}x{res} content+style, batch {batch}", "resolution": res,
                   "batch_per_gpu": batch, "global_batch": batch * world, "compute_dtype": dts,
                   "parallelism": f"replicas x{world}"},
    }


def run_video(dtype, steps, warmup, rank, world):
    """BASELINE configs[4]: infer_video.py per-frame ingest + stylisation at 1080x1920 with a 256^2
    style encoded once (its K/V cached by the AdaFormer, engine.style_cache) plus the temporal
    warping-error metric of the new frame against the previous one (exps_sintel.py:101-109,
    HIP warp kernel).  Synthetic smooth video: seeded low-frequency noise translating by a known
    (3, 1) px per frame; the flow is that translation, the mask its forward/backward check."""
    from mhada_hip import video
    from mhada_hip.recipe import seeded_image
    vc, vs, ada = build_models(dtype)
    dev = torch.device("cuda", torch.cuda.current_device())
    H, W, n = 1080, 1920, steps + warmup + 1
    g = torch.Generator(device="cpu").manual_seed(500 + rank)
    base = torch.nn.functional.interpolate(torch.rand(1, 3, H // 8 + 2, W // 8 + 2, generator=g) * 255,
                                           size=(H + 16 * n, W + 16 * n), mode="bilinear", align_corners=False)
    frames = [base[:, :, 1 * t: 1 * t + H, 3 * t: 3 * t + W].contiguous().to(dev) for t in range(n)]
    flow = torch.empty(1, 2, H, W, device=dev)
    flow[:, 0], flow[:, 1] = 3.0, 1.0  # frame t+1 at p equals frame t at p + (3, 1)
    # the stream arrives as cv2 frames: u8 BGR HWC (device-resident, like every bench input);
    # each step ingests one (utilities.cv2_to_tensor: BGR->RGB, toTensor255; HIP frame ingest),
    # stylises it against the cached style and scores the warping error against the previous one
    frames_u8 = [f[0].permute(1, 2, 0).flip(-1).round().clamp(0, 255).to(torch.uint8).contiguous() for f in frames]
    del frames
    st = video.VideoStylizer(vc, vs, ada)
    with torch.no_grad():
        st.set_style(seeded_image(1, 256, 256, 12 + 1000 * rank).to(dev))
        mask = video.flow_warp_mask(flow[0], -flow[0])
        st(video.cv2_to_tensor(frames_u8[0]).unsqueeze(0))

        def step(t):
            st(video.cv2_to_tensor(frames_u8[t]).unsqueeze(0))
            return st.warping_error(flow, mask)

        for t in range(1, warmup + 1):
            step(t)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with _mark(f"video_1080p_{'f32' if dtype == torch.float32 else 'bf16'}", steps):
            for t in range(warmup + 1, warmup + 1 + steps):
                err = step(t)
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    assert torch.isfinite(err).all()
    elapsed = max_over_ranks(elapsed, world)
    clock = shader_clock()
    nc, ns = (H // 8) * (W // 8), (256 // 8) ** 2
    d = 64
    fl = (72 * nc * C * C + 196608 * nc + 6 * (6 * nc * ns * C + 2 * nc * C * d + 2 * nc * C * C)
          + 30892032 * nc)  # SURVEY §8d, style side cached
    dts = "f32" if dtype == torch.float32 else "bf16"
    return {"value": steps * world / elapsed, "unit": "frames/s", "ms_per_frame": elapsed / steps * 1e3,
            "dtype": dts, "tflops": fl * steps / elapsed / 1e12, "warping_error_last": float(err[0]),
            "clock_ghz": clock,
            "config": {"workload": "infer_video.py: 1080x1920 u8 BGR frames -> ingest (cv2_to_tensor) -> stylise "
                                   "against a cached 256x256 style, + warping error",
                       "batch_per_gpu": 1, "compute_dtype": dts, "parallelism": f"replicas x{world}"}}


def run_infer_time(dtype, warmup, runs=100):
    """The reference's own latency probe, infer_time.py:64-87: B=1, 512^2 content + style,
    ``vit_c -> vit_s -> adaFormer -> clamp(0, 255)``, each run bracketed by its own events and a
    synchronize, averaged over 100 runs (after ``warmup`` untimed runs; the reference times its
    first run too).  Reported eager (the module calls as the reference makes them) and as one
    hipGraph replay of the same call (mhada_hip.graphs.GraphedStylizer, bit-identical output);
    1 - graph / eager = the share of the eager call that is host-side launch overhead / gaps."""
    from mhada_hip.graphs import GraphedStylizer
    from mhada_hip.recipe import seeded_image
    vc, vs, ada = build_models(dtype)
    dev = bench_device()
    c = seeded_image(1, 512, 512, 11).to(dev)
    s = seeded_image(1, 512, 512, 12).to(dev)

    def eager():
        fc = vc(c)
        fs = vs(s)
        _, cs = ada(fc, fs)
        return cs.clamp(0, 255)

    def probe(fn, tag):
        with torch.no_grad():
            for _ in range(warmup):
                fn()
            torch.cuda.synchronize()
            total = 0.0
            with _mark(f"infer_time_{'f32' if dtype == torch.float32 else 'bf16'}_{tag}", runs):
                for _ in range(runs):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    out = fn()
                    b.record()
                    torch.cuda.synchronize()
                    total += a.elapsed_time(b)
        return total / runs, out

    t_eager, ref = probe(eager, "eager")
    ref = ref.clone()
    g = GraphedStylizer(vc, vs, ada, (1, 3, 512, 512))
    t_graph, out = probe(lambda: g(c, s), "graph")
    dts = "f32" if dtype == torch.float32 else "bf16"
    return {"ms_per_frame": round(t_eager, 4), "ms_per_frame_graph": round(t_graph, 4),
            "launch_gap_share": round(1.0 - t_graph / t_eager, 4), "graph_bit_identical": bool(torch.equal(out, ref)),
            "runs": runs, "dtype": dts, "unit": "ms/frame",
            "config": {"workload": "infer_time.py: B=1 512x512 content+style, vit_c -> vit_s -> adaFormer -> clamp, "
                                   "per-run CUDA-event timing averaged over 100 runs", "batch": 1, "resolution": 512}}


def run_train(steps, warmup, rank, world, res=512, batch=8):
    """BASELINE configs[3]: train_image.py step at 512^2, 8 images per GPU, DP over RCCL.
    (res / batch are smaller only in the CPU rehearsal of the rank protocol, tests/test_bench_cpu.py.)"""
    import network
    from mhada_hip.recipe import load_recipe, seeded_image
    from mhada_hip.train import Trainer
    dev = bench_device()
    vc = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c").to(dev).train()
    vs = load_recipe(network.VisionTransformer(pos_embedding=False), "vit_s").to(dev).train()
    ada = load_recipe(network.AdaAttnTransformerMultiHead(), "ada").to(dev).train()
    vgg = load_recipe(network.VGG19(), "vgg").to(dev)
    tr = Trainer(vc, vs, ada, vgg)
    for i in range(warmup):
        tr.step(seeded_image(batch, res, res, 100 + rank * 1000 + i).to(dev),
                seeded_image(batch, res, res, 500 + rank * 1000 + i).to(dev))
    data = [(seeded_image(batch, res, res, 100 + rank * 1000 + warmup + i).to(dev),
             seeded_image(batch, res, res, 500 + rank * 1000 + warmup + i).to(dev)) for i in range(steps)]
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    with _mark(f"train_{res}_b{batch}", steps) if dev.type == "cuda" else contextlib.nullcontext():
        for c, s in data:
            last = tr.step(c, s)
        sync()
    if world > 1:
        dist.barrier()
    sync()
    el = time.perf_counter() - t0
    el = max_over_ranks(el, world)
    clock = shader_clock() if dev.type == "cuda" else None
    agree = None
    if world > 1:
        agree = rank_agreement([tr.vit_c, tr.vit_s, tr.ada])
        assert agree["identical"], f"DP ranks diverged: {agree}"
    backend = dist.get_backend() if world > 1 else None
    return {"metric": f"train_image.py step throughput at {res}x{res}, {batch} images/GPU [configs[3]]",
            "value": round(batch * steps * world / el, 3), "unit": "images/s", "n_gpus": world, "steps": steps,
            "warmup": warmup, "ms_per_step": round(el / steps * 1e3, 2), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic rand*255 images, recipe random-init weights",
            "config": {"workload": "train step (4 ViT + 3 AdaFormer + 5 VGG19 fwd, 4 losses, bwd, Adam)",
                       "global_batch": batch * world, "resolution": res, "device": dev.type,
                       "parallelism": (f"dp{world} ({'RCCL' if backend == 'nccl' else backend} grad all-reduce)"
                                       if world > 1 else "single GPU"),
                       "backend": backend,
                       "engine": ("every conv / linear / attention fwd+bwd on HIP kernels (Winograd fp32 convs, "
                                  "dS-spill attention backward, TN weight-gradient GEMMs); losses, Adam and glue on "
                                  "PyTorch-ROCm (DESIGN.md §3b)" if dev.type == "cuda" else
                                  "CPU rehearsal of the rank protocol: the reference's aten expression")},
            "last_losses": last, "rank_agreement": agree, "clock_ghz": clock}


def rank_agreement(modules) -> dict:
    """After DP steps every rank must hold bit-identical parameters (same averaged gradients, same
    Adam): per-parameter fp64 checksums, all-reduced MAX and MIN over the ranks, must coincide."""
    ps = [p for m in modules for p in m.parameters()]
    dev = ps[0].device if dist.get_backend() == "nccl" else torch.device("cpu")
    sums = torch.stack([p.detach().double().sum() for p in ps]).to(dev)
    sq = torch.stack([p.detach().double().square().sum() for p in ps]).to(dev)
    v = torch.cat([sums, sq])
    hi, lo = v.clone(), v.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    spread = float((hi - lo).abs().max())
    return {"params": len(ps), "max_checksum_spread": spread, "identical": spread == 0.0,
            "backend": dist.get_backend(), "world": dist.get_world_size()}


def cpu_model() -> str:
    import subprocess
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:  # pragma: no cover
        pass
    return "unknown"


def cpu_threads() -> tuple:
    """(threads used, CPUs in this process's affinity mask).  SURVEY §8(d): the CPU path runs with
    torch.set_num_threads(len(os.sched_getaffinity(0))); the GPU box caps a job's CPU share with
    OMP_NUM_THREADS (16 per GPU there), which bounds the count when it is smaller."""
    aff = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(aff, cap) if cap > 0 else aff), aff


def cpu_baseline():
    """The reference's PyTorch CPU arithmetic timed on the box's host cores (SURVEY §8d "CPU path
    beside it"; infer_time.py:64-87 times the same three module calls): tests/torch_ref.py — the
    aten fp32 restatement of vit_c / vit_s / adaFormer, pinned to the reference's own outputs by
    tests/test_torch_ref_cpu.py — at B=1: 5 frames at 256^2, 8 at 512^2 (the headline value: the
    median frame, since the box's host cores are shared) and one 1024^2 frame, on
    torch.set_num_threads(cores).  The numpy oracle (oracle/mhada_oracle.py)
    is timed beside it at 256^2 as a second, labelled number."""
    from mhada_hip.recipe import recipe_state_dict, seeded_image
    from oracle import mhada_oracle as O
    import network
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import torch_ref
    threads, aff = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    shapes = lambda m: {k: tuple(v.shape) for k, v in m.state_dict().items()}  # noqa: E731
    sd_vc = recipe_state_dict("vit_c", shapes(network.VisionTransformer(pos_embedding=True)))
    sd_vs = recipe_state_dict("vit_s", shapes(network.VisionTransformer(pos_embedding=False)))
    sd_ada = recipe_state_dict("ada", shapes(network.AdaAttnTransformerMultiHead()))
    per_res, oracle_res = {}, {}
    try:
        with torch.no_grad():  # one untimed small call (thread pool, allocator)
            torch_ref.stylize(seeded_image(1, 256, 256, 11), seeded_image(1, 256, 256, 12), sd_vc, sd_vs, sd_ada)
        for res, n in ((256, 5), (512, 8), (1024, 1)):
            c = seeded_image(1, res, res, 11)
            s = seeded_image(1, res, res, 12)
            ts = []
            with torch.no_grad():
                for _ in range(n):
                    t0 = time.perf_counter()
                    torch_ref.stylize(c, s, sd_vc, sd_vs, sd_ada)
                    ts.append(time.perf_counter() - t0)
            med = sorted(ts)[len(ts) // 2]  # the host cores are shared: the median frame, not the mean
            per_res[f"{res}x{res}_b1"] = {"frames_per_s": round(1.0 / med, 5), "frames": n, "seconds": round(sum(ts), 2),
                                          "median_s": round(med, 4), "min_s": round(min(ts), 4), "max_s": round(max(ts), 4)}
        p = [O.to_numpy_params(sd) for sd in (sd_vc, sd_vs, sd_ada)]
        for res, n in ((256, 2),):
            c = seeded_image(1, res, res, 11).numpy()
            s = seeded_image(1, res, res, 12).numpy()
            t0 = time.perf_counter()
            for _ in range(n):
                O.stylize(c, s, *p)
            el = time.perf_counter() - t0
            oracle_res[f"{res}x{res}_b1"] = {"frames_per_s": round(n / el, 5), "frames": n, "seconds": round(el, 2)}
    finally:
        torch.set_num_threads(prev)
    v = per_res["512x512_b1"]
    return {"value": v["frames_per_s"], "unit": "frames/s", "cores": threads, "affinity_cpus": aff, "kind": "port",
            "cpu_model": cpu_model(), "per_resolution": per_res,
            "sample": f"tests/torch_ref.py (the reference's aten fp32 expression, golden-pinned) on "
                      f"torch.set_num_threads({threads}), recipe weights, B=1: "
                      + ", ".join(f"{k} {d['frames']} frame(s) in {d['seconds']} s (median {d['median_s']} s)"
                                  for k, d in per_res.items())
                      + "; value = 1 / the median 512x512 frame time",
            "numpy_oracle": {"per_resolution": oracle_res,
                             "note": "oracle/mhada_oracle.py (numpy fp32, same weights), BLAS threads as configured"}}


def _free_port() -> int:
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int) -> int:
    """Start ranks 0..n-1 of this same command as child processes (one per GPU) and wait for them.
    Runs in a parent that has made NO GPU call (so no exec-after-GPU-init anywhere); the children
    inherit stdout (rank 0 prints the JSON line).  If a rank fails, the others are stopped (by
    their own PIDs) so a rank blocked in a collective cannot hang the job; returns the first
    non-zero exit status, else 0."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            code = procs[r].poll()
            if code is None:
                continue
            live.discard(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"bench.py: rank {r} exited with status {code}; stopping the other ranks", file=sys.stderr)
                for o in live:
                    procs[o].terminate()
                for o in live:
                    try:
                        procs[o].wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        procs[o].kill()
                        procs[o].wait()
                live.clear()
        time.sleep(0.2)
    return rc


def bench_device() -> torch.device:
    """The rank's device: its GPU, or the CPU under --device cpu (the CPU rehearsal of the
    multi-rank protocol in tests/test_bench_cpu.py; the aten path of the drop-in modules)."""
    return _DEVICE[0]


_DEVICE = [torch.device("cpu")]


def sync():
    if bench_device().type == "cuda":
        torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); > 1 without a launcher starts the ranks itself")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the 1024^2 bf16 config")
    ap.add_argument("--only-secondary", action="store_true", help="run only the 1024^2 bf16 config (profiling)")
    ap.add_argument("--train", action="store_true", help="only BASELINE configs[3]: DP training step at 512^2")
    ap.add_argument("--no-train", action="store_true", help="skip the training config in the default line")
    ap.add_argument("--device", choices=("cuda", "cpu"), default="cuda",
                    help="cpu: rehearse the rank protocol on the CPU (--train only, gloo; tests)")
    ap.add_argument("--train-res", type=int, default=512, help=argparse.SUPPRESS)
    ap.add_argument("--train-batch", type=int, default=8, help=argparse.SUPPRESS)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        if args.gpus is not None and args.gpus > 1:
            sys.exit(launch_ranks(args.gpus))  # no GPU call has happened in this process
    elif args.gpus is not None and int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("MHADA_BENCH_BACKEND", "nccl" if args.device == "cuda" else "gloo")
    if args.device == "cpu":
        if not args.train or backend != "gloo":
            raise SystemExit("bench.py --device cpu rehearses the DP training protocol only (--train, gloo)")
    else:
        ndev = torch.cuda.device_count()
        if backend == "nccl" and world > ndev:
            raise SystemExit(f"bench.py: {world} RCCL ranks but {ndev} visible GPU(s)")
        # one process per GPU; the modulo only matters for a gloo rehearsal with more ranks than
        # devices (MHADA_BENCH_BACKEND=gloo on a 1-GPU box)
        local = local % max(1, ndev)
        torch.cuda.set_device(local)
        _DEVICE[0] = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    if args.train:
        r = run_train(args.steps, args.warmup, rank, world, args.train_res, args.train_batch)
        if rank == 0:
            print(json.dumps(r), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    if args.only_secondary:
        r = run_config(1024, 4, torch.bfloat16, args.steps, args.warmup, rank, world)
        if rank == 0:
            print(json.dumps(r), flush=True)
        return
    main_cfg = run_config(512, 8, torch.float32, args.steps, args.warmup, rank, world)
    second = None if args.no_secondary else run_config(1024, 4, torch.bfloat16, args.steps, args.warmup, rank, world)
    videos = {} if args.no_secondary else {
        f"video_1080p_s256_{'f32' if dt == torch.float32 else 'bf16'}": run_video(dt, args.steps, args.warmup, rank, world)
        for dt in (torch.float32, torch.bfloat16)}
    train = None if (args.no_secondary or args.no_train) else run_train(args.steps, args.warmup, rank, world,
                                                                         args.train_res, args.train_batch)
    probes = {} if args.no_secondary else {
        f"infer_time_512_b1_{'f32' if dt == torch.float32 else 'bf16'}": run_infer_time(dt, max(args.warmup, 3))
        for dt in (torch.float32, torch.bfloat16)}

    if rank == 0:
        line = {
            "metric": "stylized frames/sec (whole job) at 512x512 batch 8 fp32 [configs[1]]",
            "value": round(main_cfg["value"], 3),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(main_cfg["ms_per_step"], 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": main_cfg["dtype"],
            "data": "synthetic rand*255 images, recipe random-init weights (no checkpoint ships)",
            "config": main_cfg["config"],
            "roofline": main_cfg["roofline"],
            "tflops_whole_step": round(main_cfg["tflops_whole_step"], 2),
            "clock_ghz": main_cfg["clock_ghz"],
        }
        if second is not None:
            line["configs"] = {"1024x1024_b4_bf16": {k: second[k] for k in
                                                    ("value", "ms_per_step", "frames_per_s_per_gpu", "dtype",
                                                     "tflops_whole_step", "roofline", "clock_ghz", "config")}}
        if videos:
            line.setdefault("configs", {}).update(videos)
        if train is not None:
            line.setdefault("configs", {})["train_512_b8_f32"] = {
                k: train[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup", "dtype", "config", "last_losses",
                                      "clock_ghz")}
        if probes:
            line.setdefault("configs", {}).update(probes)
        if not args.no_cpu_baseline:
            # rank 0 only, after every timed region (the other ranks wait at the final barrier)
            line["cpu_baseline"] = cpu_baseline()
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

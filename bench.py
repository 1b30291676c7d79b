#!/usr/bin/env python3
"""Throughput of the embedding hot path on MI355X (BASELINE.json metric).

Workload (N=1 default): BASELINE.json configs[1] — WavLM-base, bf16, batch 256 x 3 s @ 16 kHz
synthetic clips -> embeddings of hidden states [12, 11, 10, 6] (REF/WavLM_embeddings.py:506).
A "step" = one sse_embed call over the rank's batch of 256 clips (conv frontend ->
projection -> pos-conv -> 12 encoder layers -> pooling), inputs resident in HBM; with N > 1
each rank processes its own 256 clips (weak scaling, clip-sharded corpus, configs[3]) and
the step ends with one RCCL all-gather of the [256, 4, 768] fp32 embeddings.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 the driver uses
torch.distributed.run (one rank per GPU, RANK/LOCAL_RANK/WORLD_SIZE from the env).

The JSON line carries:
  value         clips/s over K steps timed without instrumentation.
  roofline      dominant kernel (most device time): algorithmic FLOPs per launch / its mean
                launch time, both from HIP events recorded around every launch on the launch
                stream (sse_profile_*) during a second timed region of the same K steps
                (profiled_ms_per_step: that region's step time, events included); traffic from
                the committed rocprofv3 PMC summary of the same workload.
  cpu_baseline  the reference's CPU path on this host's cores, a bounded sample of clips (rank 0,
                N = 1 only): WavLM = oracle/wavlm_aten.py, the reference's batch-1 loop on the same
                ATen ops, calibrated against the reference itself ("calibrated-aten",
                profiles/r2_cpu_baseline_calibration.json).
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import config as C, synth  # noqa: E402
from ssr_amd.model import SSEModel  # noqa: E402
from ssr_amd.corpus import StepGather  # noqa: E402

# Algorithmic FLOPs per clip: 2 x MACs of every GEMM/conv + QK^T, AV.
FLOP_PER_CLIP = {"wavlm-base": 42.39e9, "wavlm-large": 109.6e9, "whisper-large-v2": 2272.67e9,
                 "whisper-small": 344.16e9}   # whisper-small: conv 6.41 + 12 x 28.15 (attention 6.91) GF
# MI355X dense MFMA peaks (MI355X_MICROARCH.md); fp16x3 runs three fp16 products per logical
# multiply-add, so its model-level peak is the fp16 (= bf16) peak / 3 (its GEMM roofline counts the MFMA work)
PEAK_TFLOPS = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 157.3, "fp8": 5000.0, "fp16x3": 2500.0 / 3}
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="wavlm-base",
                    choices=["wavlm-base", "wavlm-large", "whisper-large-v2", "whisper-small"],
                    help="wavlm-large: the reference's default --model_name (REF/WavLM_embeddings.py:34); "
                         "whisper-small: the default of REF/whisper_embeddings_large.py:34")
    ap.add_argument("--batch", type=int, default=None,
                    help="clips per rank per step (default 256 WavLM / 64 Whisper bf16 / 128 Whisper fp8)")
    ap.add_argument("--seconds", type=float, default=None, help="clip length (default 3 s / 30 s)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp8", "fp16x3", "fp16"],
                    help="fp8: Whisper only, MX-fp8 QKV / fc1 / fc2 GEMMs (BASELINE configs[4]); fp16x3: "
                         "WavLM / Whisper, split-fp16 GEMMs, fp32-class (<= 1e-4) embeddings; fp16: WavLM, the bf16 "
                         "path with fp16 activations / operands (same MFMA rate, 8 more mantissa bits)")
    ap.add_argument("--cpu-sample", type=int, default=None, help="clips for the CPU baseline (0 = skip)")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-launch event timing")
    ap.add_argument("--stream", action="store_true",
                    help="clips streamed from pinned host memory each step (double-buffered H2D on a side stream)")
    ap.add_argument("--logmel", action="store_true",
                    help="the Whisper log-mel front end alone (sse_logmel, K9): B x 30 s clips -> [B, 80, 3000], "
                         "reported against the HBM roofline (1.92 MB in + 0.96 MB out per clip) with the STFT "
                         "kernel's PMC-measured VALU issue / wait fractions (roofline.valu)")
    ap.add_argument("--lib", default=None, help="load this build of libsse.so instead of the in-tree one (A/B)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="sse_set_option A/B kernel switch (repeatable)")
    ap.add_argument("--corpus", type=int, default=0,
                    help="BASELINE configs[3] mode: embed a corpus of this many clips (e.g. 50000) sharded "
                         "across the ranks with corpus.extract_corpus (tail batch + one all-gather timed)")
    ap.add_argument("--corpus-resident", action="store_true",
                    help="--corpus with the clips already in HBM (default: staged from pinned host memory)")
    ap.add_argument("--ragged", action="store_true",
                    help="--corpus with mixed clip lengths (1 s .. --seconds), ragged batches")
    return ap.parse_args()


def host_threads() -> int:
    """CPU threads this process may use: its affinity set, capped by OMP_NUM_THREADS when the host
    sets one (the GPU box gives each 1-GPU job a 16-CPU share of a 256-CPU machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(omp))) if omp.isdigit() and int(omp) > 0 else n


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


CALIBRATION = "profiles/r4_cpu_baseline_calibration_wavlm.json"   # 16 clips x 7 alternating rounds
CALIBRATION_WHISPER = "profiles/r4_cpu_baseline_calibration_whisper.json"   # encoder-only, 8 clips x 5 rounds
LOGMEL_PMC = "profiles/r4_pmc_sq_logmel_b128.json"            # SQ counters of the log-mel kernels, B = 128
LOGMEL_TRAFFIC = "profiles/r4_pmc_traffic_logmel_b128.json"    # FETCH / WRITE_SIZE of the same


def cpu_baseline(model_name: str, n: int, seconds: float):
    """The reference's CPU path timed on this host's cores (rank 0, N = 1).  WavLM: the ATen
    restatement oracle/wavlm_aten.py (the reference's batch-1 loop on the same torch ops as HF
    WavLMModel), calibrated against the reference itself (oracle/calibrate_cpu_baseline.py).
    Test infrastructure, used only as the reported baseline."""
    if model_name.startswith("wavlm"):
        from oracle.wavlm_aten import WavLMAten
        thr = host_threads()
        torch.set_num_threads(thr)
        spec = C.WAVLM_BASE if model_name == "wavlm-base" else C.WAVLM_LARGE
        o = WavLMAten(spec, synth.synth_wavlm_state_dict(spec, seed=7))
        clips = synth.synth_clips(n + 1, int(16000 * seconds), seed=2024)
        idx = spec.default_layer_indices()
        o.extract(clips[0], idx)                                     # warm-up (threads, page-in)
        t0 = time.perf_counter()
        for c in clips[1:]:
            o.extract(c, idx)
        dt = time.perf_counter() - t0
        cal = None
        if os.path.exists(os.path.join(ROOT, CALIBRATION)):
            with open(os.path.join(ROOT, CALIBRATION)) as fh:
                cal = json.load(fh)
        return {"value": round(n / dt, 4), "unit": "clips/s", "cores": thr, "kind": "calibrated-aten",
                "calibration_ratio": cal and cal["ratio"], "calibration_source": cal and CALIBRATION,
                "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
                "sample": f"{n} synthetic {seconds:g} s clips, batch-1 loop of oracle/wavlm_aten.py (the reference's "
                          f"fp32 ATen ops, torch.set_num_threads({thr})), {dt:.1f} s"}
    # Whisper: oracle/whisper_aten.py, the reference's extract_whisper_embeddings_fixed on the same ATen
    # ops (log-mel via torch.stft, HF WhisperEncoder's convs / addmm / SDPA / LayerNorm), batch-1,
    # calibrated against the reference itself, like for like (oracle/calibrate_cpu_baseline.py --model
    # whisper-large-v2: the reference's model with decoder_layers = 0, so its 1-token decoder pass is one
    # embedding row; round 4).  Timed here on the encoder part only: the GPU line measures encoder
    # embeddings (BASELINE configs[2] / [4]).
    from oracle.whisper_aten import WhisperAten
    thr = host_threads()
    torch.set_num_threads(thr)
    spec = C.WHISPER_SMALL if model_name == "whisper-small" else C.WHISPER_LARGE_V2
    o = WhisperAten(spec, synth.synth_whisper_state_dict(spec, seed=11))
    clips = synth.synth_clips(n + 1, int(16000 * seconds), seed=2024)
    idx = spec.default_layer_indices()
    o.extract(clips[0], idx)                                         # warm-up
    t0 = time.perf_counter()
    for c in clips[1:]:
        o.extract(c, idx)
    dt = time.perf_counter() - t0
    cal = None
    if os.path.exists(os.path.join(ROOT, CALIBRATION_WHISPER)):
        with open(os.path.join(ROOT, CALIBRATION_WHISPER)) as fh:
            cal = json.load(fh)
    return {"value": round(n / dt, 4), "unit": "clips/s", "cores": thr, "kind": "calibrated-aten",
            "calibration_ratio": cal and cal["ratio"], "calibration_source": cal and CALIBRATION_WHISPER,
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "sample": f"{n} synthetic {seconds:g} s clips, batch-1 loop of oracle/whisper_aten.py (the reference's "
                      f"fp32 ATen ops: log-mel + encoder + time-means; torch.set_num_threads({thr})), {dt:.1f} s"}


# rocprofv3 PMC traffic per kernel (tools/pmc_traffic.sh: FETCH_SIZE x2 + WRITE_SIZE per launch),
# measured on the same workload; kernel symbols of each bench tag prefix
TRAFFIC_FILE = {("wavlm-base", "bf16"): "profiles/r6_pmc_traffic_wavlm_base_bf16_final2.json",
                ("whisper-large-v2", "fp8"): "profiles/r6_pmc_traffic_whisper_large_v2_fp8_final2.json"}
TAG_SYMBOLS = {"gemm": ("gemm8_kernel<0, false, false, false>", "gemm8p_kernel", "gemm8r_kernel"),
               # (round 5: the compile-time epilogue forms gemm8_kernel<0, true, false, true, MXE>)
               "gemm_mx": ("gemm8_kernel<0, true, false, true", "gemm8_kernel<0, false, false, true"),
               "attn": ("attention_",), "attn_f8": ("attention_f8",),
               "conv0_gn": ("conv0_mfma", "conv0_moments", "gn_finalize")}


def pmc_traffic(model_name, dtype, kernel, launch_counts):
    """Launch-weighted mean HBM bytes per launch of the kernels behind a bench tag, or None."""
    path = TRAFFIC_FILE.get((model_name, dtype))
    if not path or not os.path.exists(os.path.join(ROOT, path)):
        return None, None
    with open(os.path.join(ROOT, path)) as fh:
        ks = json.load(fh)["kernels"]
    pats = TAG_SYMBOLS.get(kernel, (kernel,))
    sel = [v for k, v in ks.items() if any(p in k for p in pats)]
    n = sum(v["launches"] for v in sel)
    if not n:
        return None, path
    return sum(v["hbm_bytes_per_launch"] * v["launches"] for v in sel) / n, path


def roofline(records, dtype):
    """Dominant kernel over the timed region: the kernel symbol (tag prefix) with most time."""
    by_kernel = {}
    for tag, ms, fl, by in records:
        k = tag.split(":", 1)[0]
        d = by_kernel.setdefault(k, [0.0, 0.0, 0.0, 0])
        d[0] += ms
        d[1] += fl
        d[2] += by
        d[3] += 1
    total = sum(v[0] for v in by_kernel.values())
    name, (ms, fl, by, n) = max(by_kernel.items(), key=lambda kv: kv[1][0])
    achieved = fl / (ms * 1e-3) / 1e12
    # the MX-fp8 GEMM is priced at the dense fp8 peak, every other kernel at the bf16 (fp32) one
    peak = PEAK_TFLOPS["fp8"] if name == "gemm_mx" else PEAK_TFLOPS["fp32" if dtype == "fp32" else "bf16"]
    mfma_work = 1.0
    if dtype == "fp16x3" and name == "gemm":   # split-fp16: three fp16 products per logical multiply-add
        mfma_work = 3.0
        achieved *= 3.0
    breakdown = {k: {"ms": round(v[0], 3), "launches": v[3], "share": round(v[0] / total, 4),
                     "tflops": round(v[1] / max(v[0], 1e-9) / 1e9, 1)} for k, v in sorted(by_kernel.items())}
    by_role = {}
    for tag, t_ms, t_fl, _ in records:
        d = by_role.setdefault(tag, [0.0, 0.0, 0])
        d[0] += t_ms
        d[1] += t_fl
        d[2] += 1
    roles = {k: {"ms": round(v[0], 3), "launches": v[2], "tflops": round(v[1] / max(v[0], 1e-9) / 1e9, 1)}
             for k, v in sorted(by_role.items())}
    return {"bound": "mfma", "kernel": name, "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": None, "mfma_work_per_flop": mfma_work,
            "alg_bytes_per_launch": by / n, "flop_per_launch": fl / n, "mean_launch_ms": round(ms / n, 4), "launches": n,
            "device_ms_per_step_sum": None, "breakdown": breakdown, "roles": roles}


def logmel_run(a, dev):
    """K9 alone: sse_logmel over a resident batch of 30 s clips (REF/whisper_embeddings_large.py:242-246,
    HF WhisperFeatureExtractor).  Algorithmic HBM bytes per clip: 480000 fp32 samples in + 80 x 3000
    fp32 log-mel out; time per call from torch events around the timed calls (one stream)."""
    from ssr_amd.model import logmel
    B = a.batch or 128
    L = 480000
    clips = torch.from_numpy(synth.synth_clips(B, L, seed=1234)).to(dev)
    for _ in range(a.warmup):
        logmel(clips)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(a.steps):
        out = logmel(clips)
    e1.record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ms = e0.elapsed_time(e1) / a.steps
    # algorithmic HBM bytes: the clip read once, the 80 x 3000 fp32 output written once (the fused
    # kernel also writes and re-reads its [3000][80] fp32 log-mel scratch before the per-clip max
    # clamp: real traffic = by + 2 x 0.96 MB per clip)
    by = B * (L * 4.0 + 80 * 3000 * 4.0)
    gbs = by / (ms * 1e-3) / 1e9
    # what actually bounds the STFT kernel: its SQ counters (tools/pmc_kernel.sh, committed file) give the
    # VALU issue fraction (wave-64 VALU instructions x 2 cycles over 1024 SIMDs x the kernel's cycles per
    # XCD) and the share of wave cycles spent waiting (s_waitcnt / barriers); HBM traffic from the PMC
    # traffic file when present
    valu = None
    try:
        with open(os.path.join(ROOT, LOGMEL_PMC)) as fh:
            pm = json.load(fh)
        k = next(k for k in pm if "lm_stft_mel" in k)
        c = {n: v["mean"] for n, v in pm[k].items()}
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0
        valu = {"kernel": k.replace("(anonymous namespace)::", "").split("(")[0], "valu_insts_per_call": c["SQ_INSTS_VALU"],
                "valu_issue_frac": round(c["SQ_INSTS_VALU"] * 2.0 / (1024 * cyc), 3),
                "lds_insts_per_call": c["SQ_INSTS_LDS"],
                "wait_frac_of_wave_cycles": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3),
                "lds_bank_conflict_cycles": c["SQ_LDS_BANK_CONFLICT"], "source": LOGMEL_PMC,
                "reading": "neither HBM- nor VALU-bound: latency (LDS round trips between the FFT stages' "
                           "wave barriers) -- the issue fraction is the headroom a deeper schedule could use"}
    except (OSError, StopIteration, KeyError, ValueError):
        pass
    traffic = None
    try:
        with open(os.path.join(ROOT, LOGMEL_TRAFFIC)) as fh:
            tj = json.load(fh)
        traffic = sum(v["hbm_bytes_per_launch"] for k, v in tj["kernels"].items() if "lm_" in k)
    except (OSError, KeyError, ValueError):
        pass
    res = {"metric": "clips/sec (30 s) Whisper log-mel front end", "value": round(B * a.steps / el, 1), "unit": "clips/s",
           "n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(1e3 * el / a.steps, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic 16 kHz clips (splitmix64 Gaussian+tones)",
           "config": {"workload": f"log-mel of {B} x 30 s clips -> [{B}, 80, 3000] fp32 (sse_logmel)", "global_batch": B},
           "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "alg_bytes_per_call": by,
                        "mean_call_ms": round(ms, 4), "valu": valu,
                        "note": "fused STFT (LDS FFT) + |X|^2 + mel + log10 per 20-frame block, then the per-clip "
                                "max clamp; the spectrum never leaves LDS"},
           "finite": bool(torch.isfinite(out).all().item())}
    print(json.dumps(res), flush=True)


def corpus_run(a, model, spec, idx, clips, B, L, world, rank, dev, dist):
    """configs[3]: the whole corpus through corpus.extract_corpus (rank r embeds its contiguous
    shard in batches of B, then ONE all-gather assembles [N, n_layers, H] in corpus order).  The
    synthetic corpus cycles the rank's B distinct clips (every clip is still embedded), held in
    pinned HOST memory: each batch is copied to the device on extract_corpus's side stream while the
    previous one computes, so the host staging SURVEY §8(e) names as the scaling limiter is inside
    the timed region (--corpus-resident: clips already in HBM).  --ragged: clip lengths drawn in
    [1 s, L] (sorted per batch, embedded at their own lengths through sse_embed_ragged).
    Warm-up: one full pass; timed: a second pass, barrier + sync on both sides."""
    from ssr_amd.corpus import extract_corpus, sse_embed_fn
    N = a.corpus
    host = clips.cpu().pin_memory()
    lens_all = None
    if a.ragged:
        rng = np.random.default_rng(77 + rank)
        lens_all = np.sort(rng.integers(16000, L + 1, size=B)).tolist()

    def source(s, e):
        if a.corpus_resident:
            r = torch.arange(s, e, device=dev) % B
            w = clips.index_select(0, r)
        else:
            o = s % B                      # s is a multiple of B: a pinned contiguous slice
            w = host[o:o + (e - s)]
        if lens_all is None:
            return w
        ln = [lens_all[(s + i) % B] for i in range(e - s)]
        return w[:, :max(ln)], ln

    fn = sse_embed_fn(model, idx)
    run = lambda: extract_corpus(source, N, fn, (len(idx), spec.hidden), device=dev, batch=B)
    emb = run()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    emb = run()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max = float(t.item())
    per = -(-N // world)
    if rank == 0:
        where = "HBM-resident" if a.corpus_resident else "pinned host memory, double-buffered H2D on a side stream"
        shape = (f"mixed lengths 1-{L / 16000:g} s (ragged batches)" if a.ragged else f"{L / 16000:g} s")
        res = {"metric": "clips/sec (3 s@16 kHz) embedding extraction", "value": round(N / t_max, 2), "unit": "clips/s",
               "n_gpus": world, "steps": -(-per // B), "warmup": 1, "ms_per_step": round(1e3 * t_max / -(-per // B), 3),
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": a.dtype,
               "data": f"synthetic corpus of {N} clips, {shape} (each rank cycles {B} distinct clips from {where})",
               "config": {"workload": f"{spec.name} {a.dtype} embeddings of a {N}-clip corpus, clip-sharded over "
                                      f"{world} rank(s), batches of {B}, one RCCL all-gather of [N,{len(idx)},{spec.hidden}]",
                          "model": spec.name, "global_batch": N, "clip_samples": L, "layers_pooled": idx,
                          "parallelism": f"clip-sharded dp{world}", "staging": where},
               "finite": bool(torch.isfinite(emb).all().item()), "rows": int(emb.shape[0])}
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main():
    a = parse()
    if a.lib:
        from ssr_amd import _lib
        _lib.use_library(a.lib)
    for kv in a.opt:
        from ssr_amd import _lib
        name, val = kv.split("=")
        _lib.check(_lib.lib().sse_set_option(name.encode(), int(val)), "sse_set_option " + name)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("for --gpus > 1 launch with torch.distributed.run (one process per GPU)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if a.logmel:
        return logmel_run(a, dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    wavlm = a.model.startswith("wavlm")
    spec = {"wavlm-base": C.WAVLM_BASE, "wavlm-large": C.WAVLM_LARGE, "whisper-large-v2": C.WHISPER_LARGE_V2,
            "whisper-small": C.WHISPER_SMALL}[a.model]
    if a.dtype == "fp8" and wavlm:
        raise SystemExit("--dtype fp8 is the Whisper encoder mode (BASELINE configs[4])")
    B = a.batch or (256 if wavlm else (128 if a.dtype == "fp8" else 64))
    secs = a.seconds or (3.0 if wavlm else 30.0)
    L = int(16000 * secs)
    sd = synth.synth_state_dict(spec)
    # fp16-range dtypes: no per-call range check (a host sync) inside the timed loops; one check after them
    model = SSEModel(spec, sd, device=dev, dtype=a.dtype, check_range=False)
    del sd
    idx = spec.default_layer_indices()
    clips = torch.from_numpy(synth.synth_clips(B, L, seed=1234, first_clip=rank * B)).to(dev)
    if a.corpus:
        return corpus_run(a, model, spec, idx, clips, B, L, world, rank, dev, dist)

    # --stream (configs[4] "streaming extraction"): each step's clips come from pinned host memory,
    # copied on a side stream into the other of two device buffers while this step computes
    # (double-buffered H2D; the next batch's copy waits only for the step that last read its buffer)
    if a.stream:
        host = [torch.from_numpy(synth.synth_clips(B, L, seed=1234 + k, first_clip=rank * B)).pin_memory()
                for k in range(2)]
        dbuf = [clips, torch.empty_like(clips)]
        cs = torch.cuda.Stream(device=dev)
        ready = [torch.cuda.Event(), torch.cuda.Event()]
        done = [torch.cuda.Event(), torch.cuda.Event()]
        for e in done:
            e.record()
        with torch.cuda.stream(cs):
            dbuf[0].copy_(host[0], non_blocking=True)
            ready[0].record(cs)
        it = [0]

    def embed_into(out):
        if a.stream:
            cur, nxt = it[0] % 2, (it[0] + 1) % 2
            it[0] += 1
            cs.wait_event(done[nxt])
            with torch.cuda.stream(cs):
                dbuf[nxt].copy_(host[nxt], non_blocking=True)
                ready[nxt].record(cs)
            torch.cuda.current_stream(dev).wait_event(ready[cur])
            model.embed(dbuf[cur], idx, out=out)
            done[cur].record()
        else:
            model.embed(clips, idx, out=out)

    # two output slots: step k's all-gather (RCCL, async on its own stream) overlaps step k+1's compute
    # (corpus.StepGather; its gloo twin is tests/test_corpus_dist.py::test_step_gather_*)
    pipe = StepGather(embed_into, (B, len(idx), spec.hidden), world, dev, dist)
    step, drain = pipe.step, pipe.drain

    for _ in range(a.warmup):
        step()
    drain()
    torch.cuda.synchronize()

    def timed(profile):
        """K steps between barriers + device syncs; with profile, HIP events around every launch."""
        if profile:
            # per-launch timing runs single-stream: with the two-stream half-batch split (WavLM,
            # split_forward in sse_model.hip) launches of the two halves overlap and each event pair
            # would time a shared chip; the roofline is the kernels' own rate, alone on the chip
            from ssr_amd import _lib
            prev_split = _lib.lib().sse_set_option(b"no_split", 1)
            model.profile_start(max_launches=200 * max(a.steps, 1))
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        drain()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        el = time.perf_counter() - t0
        recs = []
        if profile:
            recs = model.profile_read()
            model.profile_stop()
            _lib.lib().sse_set_option(b"no_split", prev_split)
        return el, recs

    # value: an unperturbed timed region (per-launch event records add ~0.5 ms/step of launch
    # gaps); roofline: a second timed region of the same K steps with the events (single-stream)
    elapsed, _ = timed(False)
    # N > 1: the last step's gathered [world*B, 4, H] slot checked against every rank's own rows (rank-tagged
    # clips), and the world size RCCL itself reports -- outside the timed region
    gather_check = pipe.verify() if dist is not None else None
    if gather_check is not None and gather_check["rccl_world"] != world:
        raise RuntimeError(f"RCCL world {gather_check['rccl_world']} != WORLD_SIZE {world}")
    records, prof_elapsed = [], None
    if not a.no_profile:
        prof_elapsed, records = timed(True)
    model.check_range_now()   # fp16 / fp16x3: raises SSERangeError if any timed step overflowed
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max = float(t.item())
    clips_total = world * B * a.steps
    value = clips_total / t_max

    if rank == 0:
        res = {
            "metric": "clips/sec (3 s@16 kHz) embedding extraction" if wavlm else "clips/sec (30 s) embedding extraction",
            "value": round(value, 2), "unit": "clips/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(1e3 * t_max / a.steps, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": a.dtype,
            "data": "synthetic 16 kHz clips (splitmix64 Gaussian+tones), random-init weights of the real architecture"
                    + ("; clips streamed from pinned host memory every step (double-buffered H2D)" if a.stream else ""),
            "config": {"workload": f"{spec.name} {a.dtype} embeddings, {B} x {secs:g} s clips per GPU per step"
                                   + (", RCCL all-gather of [B,4,H] per step" if world > 1 else ""),
                       "model": spec.name, "global_batch": world * B, "clip_samples": L,
                       "layers_pooled": idx, "parallelism": f"clip-sharded dp{world}"},
        }
        if gather_check is not None:
            res["rccl_world"] = gather_check["rccl_world"]
            res["gather_check"] = gather_check
        if records:
            rf = roofline(records, a.dtype)
            rf["device_ms_per_step_sum"] = round(sum(r[1] for r in records) / a.steps, 3)
            rf["profiled_ms_per_step"] = round(1e3 * prof_elapsed / a.steps, 3)
            tr, src = pmc_traffic(spec.name, a.dtype, rf["kernel"], None)
            if tr is not None:
                rf["traffic"] = round(tr)
                rf["traffic_source"] = src + " (rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE, bytes per launch)"
            res["roofline"] = rf
        res["model_flops_frac"] = round(value / world * FLOP_PER_CLIP[a.model] / 1e12 / PEAK_TFLOPS[a.dtype], 4)
        if a.dtype == "fp16x3":   # the same logical FLOPs against the dense fp16 MFMA peak (3 products per term)
            res["logical_flops_frac_dense_fp16"] = round(value / world * FLOP_PER_CLIP[a.model] / 1e12 / PEAK_TFLOPS["fp16"], 4)
        ncpu = a.cpu_sample if a.cpu_sample is not None else (256 if wavlm else 2)   # ~10-30 s of CPU work
        if world == 1 and ncpu > 0:
            res["cpu_baseline"] = cpu_baseline(a.model, ncpu, secs)
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

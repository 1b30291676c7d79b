#!/usr/bin/env python3
"""ORACLE tooling (container only): calibrate bench.py's CPU baseline against the reference itself.

Times, in this container, on the same clips, weights and thread count:
  * the reference's own ``extract_wavlm_embeddings`` (REF/WavLM_embeddings.py:267-341) on an HF
    ``WavLMModel`` (imported the way tests/golden/make_golden.py does: torchaudio stub, temp cwd,
    no bytecode written under /root/reference), batch-1 loop over ``N`` clips (REF :578-586);
  * ``oracle/wavlm_aten.py`` (the ATen restatement bench.py times on the GPU box).
The two are run in alternating rounds and each rate is the median over rounds.  The ratio
restatement / reference must lie in [0.9, 1.1]; the result goes to
profiles/r2_cpu_baseline_calibration.json (bench.py copies the ratio into its cpu_baseline).

Whisper (``--model whisper-large-v2``): the reference's ``extract_whisper_embeddings_fixed``
(REF/whisper_embeddings_large.py:234-299: log-mel, encoder, 1-token decoder) on an HF Whisper-large-v2
``WhisperModel`` vs ``oracle/whisper_aten.py``; result in profiles/r3_cpu_baseline_calibration_whisper.json.

Usage: python oracle/calibrate_cpu_baseline.py [--model wavlm-base|whisper-large-v2] [--clips 16]
       [--rounds 5] [--threads 8]   (round 4: Whisper --clips 8 --rounds 5, WavLM --rounds 7)
"""
from __future__ import annotations

import argparse
import importlib
import importlib.util
import json
import os
import platform
import statistics
import subprocess
import sys
import tempfile
import time

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


def cpu_model() -> str:
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--model", default="wavlm-base", choices=["wavlm-base", "whisper-large-v2"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.out is None:
        a.out = os.path.join(ROOT, "profiles", "r2_cpu_baseline_calibration.json" if a.model == "wavlm-base"
                             else "r3_cpu_baseline_calibration_whisper.json")
    if a.model != "wavlm-base":
        return whisper(a)

    spec_mg = importlib.util.spec_from_file_location("make_golden", os.path.join(ROOT, "tests", "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec_mg)
    spec_mg.loader.exec_module(mg)          # imports torch + transformers first (stub order)
    import numpy as np
    import torch
    from transformers import Wav2Vec2FeatureExtractor, WavLMConfig, WavLMModel
    from ssr_amd import config as C, synth
    from oracle.wavlm_aten import WavLMAten

    torch.set_num_threads(a.threads)
    spec = C.WAVLM_BASE
    sd = synth.synth_wavlm_state_dict(spec, seed=7)
    model = WavLMModel(WavLMConfig())
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    model.eval()
    fe = Wav2Vec2FeatureExtractor(do_normalize=False)
    aten = WavLMAten(spec, sd)
    clips = synth.synth_clips(a.clips + 1, 48000, seed=2024)
    idx = spec.default_layer_indices()
    paths = mg._register("calib", clips)

    cwd = os.getcwd()
    ref_rates, port_rates, max_rel = [], [], 0.0
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)
        try:
            mg._install_torchaudio_stub()
            ref = mg._import_ref("ref_wavlm_embeddings", "WavLM_embeddings.py")
            ref.extract_wavlm_embeddings(paths[0], model, fe, "cpu", idx)       # warm-up both
            aten.extract(clips[0], idx)
            for _ in range(a.rounds):
                t0 = time.perf_counter()
                got_ref = [ref.extract_wavlm_embeddings(p, model, fe, "cpu", idx) for p in paths[1:]]
                ref_rates.append(a.clips / (time.perf_counter() - t0))
                t0 = time.perf_counter()
                got = [aten.extract(c, idx) for c in clips[1:]]
                port_rates.append(a.clips / (time.perf_counter() - t0))
                for d0, d1 in zip(got_ref, got):
                    for k in d0:
                        max_rel = max(max_rel, float(np.linalg.norm(d1[k] - d0[k]) / np.linalg.norm(d0[k])))
        finally:
            os.chdir(cwd)
    r_ref, r_port = statistics.median(ref_rates), statistics.median(port_rates)
    spread = lambda v: round((max(v) - min(v)) / statistics.median(v), 4)
    res = {"reference_clips_per_s": round(r_ref, 3), "restatement_clips_per_s": round(r_port, 3),
           "spread_reference": spread(ref_rates), "spread_restatement": spread(port_rates),
           "ratio": round(r_port / r_ref, 4), "rounds_reference": [round(x, 3) for x in ref_rates],
           "rounds_restatement": [round(x, 3) for x in port_rates], "threads": a.threads,
           "host_cpus": os.cpu_count(), "cpu_model": cpu_model(), "clips": a.clips, "clip_s": 3.0,
           "max_rel_l2_restatement_vs_reference": max_rel, "torch": torch.__version__,
           "what": "REF/WavLM_embeddings.py:267-341 extract_wavlm_embeddings (HF WavLMModel, fp32, batch-1 loop) "
                   "vs oracle/wavlm_aten.py on the same clips / weights / threads, alternating rounds, medians"}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))
    if not 0.9 <= res["ratio"] <= 1.1:
        raise SystemExit(f"calibration ratio {res['ratio']} outside [0.9, 1.1]")


def whisper(a):
    """Whisper-large-v2 vs oracle/whisper_aten.py, like for like with bench.py's Whisper line (encoder
    embeddings only): the reference always runs its 1-token decoder pass
    (REF/whisper_embeddings_large.py:257-262), so its model here has decoder_layers = 0 -- the pass is then
    the token embedding + the decoder's final LayerNorm on one row, microseconds -- and the restatement
    times its encoder path only.  Encoder embeddings are compared for parity."""
    spec_mg = importlib.util.spec_from_file_location("make_golden", os.path.join(ROOT, "tests", "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec_mg)
    spec_mg.loader.exec_module(mg)
    import numpy as np
    import torch
    from transformers import WhisperConfig, WhisperFeatureExtractor, WhisperModel
    from ssr_amd import config as C, synth
    from oracle.whisper_aten import WhisperAten

    torch.set_num_threads(a.threads)
    spec = C.WHISPER_LARGE_V2
    sd = synth.synth_whisper_state_dict(spec, seed=11, full_hf=True)
    cfg = WhisperConfig(d_model=spec.d_model, encoder_layers=spec.layers, encoder_attention_heads=spec.heads,
                        decoder_layers=spec.decoder_layers, decoder_attention_heads=spec.heads,
                        encoder_ffn_dim=spec.ffn, decoder_ffn_dim=spec.dec_ffn_dim, num_mel_bins=spec.n_mels,
                        vocab_size=spec.vocab_size, max_target_positions=spec.max_target_positions)
    with torch.device("meta"):
        model = WhisperModel(cfg)
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False,
                                                assign=True)
    assert not unexpected, unexpected
    with torch.no_grad():   # decoder_layers = 0: only its token / position embeddings and final LN remain
        for name, p_ in list(model.named_parameters()):
            if p_.is_meta:
                parent = model.get_submodule(name.rsplit(".", 1)[0])
                setattr(parent, name.rsplit(".", 1)[1],
                        torch.nn.Parameter(torch.ones(p_.shape) if name.endswith("layer_norm.weight")
                                           else torch.zeros(p_.shape)))
    model.eval()
    proc = WhisperFeatureExtractor(feature_size=spec.n_mels)
    aten = WhisperAten(spec, sd)
    clips = synth.synth_clips(a.clips + 1, 48000, seed=2024)
    enc_idx, dec_idx = spec.default_layer_indices(), []
    paths = mg._register("calibw", clips)
    cwd = os.getcwd()
    ref_rates, port_rates, max_rel = [], [], 0.0
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)
        try:
            mg._install_torchaudio_stub()
            ref = mg._import_ref("ref_whisper_embeddings", "whisper_embeddings_large.py")
            ref.extract_whisper_embeddings_fixed(paths[0], model, proc, "cpu", enc_idx, dec_idx)   # warm-up both
            aten.extract(clips[0], enc_idx, dec_idx)
            for _ in range(a.rounds):
                t0 = time.perf_counter()
                got_ref = [ref.extract_whisper_embeddings_fixed(p, model, proc, "cpu", enc_idx, dec_idx) for p in paths[1:]]
                ref_rates.append(a.clips / (time.perf_counter() - t0))
                t0 = time.perf_counter()
                got = [aten.extract(c, enc_idx) for c in clips[1:]]
                port_rates.append(a.clips / (time.perf_counter() - t0))
                for d0, d1 in zip(got_ref, got):
                    for k in d1:
                        max_rel = max(max_rel, float(np.linalg.norm(d1[k] - d0[k]) / np.linalg.norm(d0[k])))
        finally:
            os.chdir(cwd)
    r_ref, r_port = statistics.median(ref_rates), statistics.median(port_rates)
    spread = lambda v: round((max(v) - min(v)) / statistics.median(v), 4)
    res = {"reference_clips_per_s": round(r_ref, 4), "restatement_clips_per_s": round(r_port, 4),
           "spread_reference": spread(ref_rates), "spread_restatement": spread(port_rates),
           "ratio": round(r_port / r_ref, 4), "rounds_reference": [round(x, 4) for x in ref_rates],
           "rounds_restatement": [round(x, 4) for x in port_rates], "threads": a.threads,
           "host_cpus": os.cpu_count(), "cpu_model": cpu_model(), "clips": a.clips, "clip_s": 3.0,
           "max_rel_l2_restatement_vs_reference": max_rel, "torch": torch.__version__,
           "what": "REF/whisper_embeddings_large.py:234-299 extract_whisper_embeddings_fixed (HF WhisperModel "
                   "large-v2 encoder, decoder_layers = 0 so the reference's 1-token decoder pass is one embedding row "
                   "+ LayerNorm; fp32, batch-1 loop) vs oracle/whisper_aten.py encoder-only (what bench.py times) on "
                   "the same clips / weights / threads, alternating rounds, medians; spread = (max - min) / median"}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))
    if not 0.9 <= res["ratio"] <= 1.1:
        raise SystemExit(f"calibration ratio {res['ratio']} outside [0.9, 1.1]")


if __name__ == "__main__":
    main()

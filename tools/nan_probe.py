"""Which path makes non-finite WavLM-base bf16 embeddings: per-layer finiteness of hidden_states for the
default configuration and with single library options flipped (debug aid)."""
import sys

import torch

import importlib  # noqa: E402

sys.path.insert(0, ".")
importlib.import_module("stuttering-speech-representation_amd")   # registers `ssr_amd`
from ssr_amd import _lib, config as C, synth  # noqa: E402
from ssr_amd.model import SSEModel  # noqa: E402


def report(tag, m, w):
    hs = m.hidden_states(w)
    bad = [i for i, h in enumerate(hs) if not torch.isfinite(h).all()]
    e = m.embed(w, list(range(13)))
    print(f"{tag:28s} non-finite hidden_states layers {bad[:6]}{'...' if len(bad) > 6 else ''}; "
          f"embed finite {bool(torch.isfinite(e).all())}", flush=True)


def main():
    sd = synth.synth_wavlm_state_dict(C.WAVLM_BASE)
    w = torch.from_numpy(synth.synth_clips(6, 48000, seed=31)).cuda()
    for dt in ("bf16", "fp16", "fp32"):
        m = SSEModel(C.WAVLM_BASE, sd, device="cuda:0", dtype=dt)
        report(f"{dt} default", m, w)
        if dt == "bf16":
            for opt in ("gemm_nonpersist", "no_lnfold", "gemm_cfg", "conv0_valu", "gelu_exact"):
                with _lib.option(opt, 1):
                    report(f"{dt} {opt}=1", m, w)
        del m


if __name__ == "__main__":
    main()

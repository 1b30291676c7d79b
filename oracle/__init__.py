"""ORACLE — TEST INFRASTRUCTURE ONLY.

A from-scratch numpy restatement of the reference's hot path:
WavLM-base/large and Whisper-encoder forward passes, the Whisper log-mel front end,
and the per-layer mean pooling of ``extract_wavlm_embeddings`` /
``extract_whisper_embeddings_fixed``.  Each function cites the reference (REF/...) or
third-party transformers 5.15.0 (HF/...) file:line it restates.

Parity pinning: the reference has no tests or golden vectors of its own.
The oracle is pinned against fixtures produced by running the reference's OWN glue
(`REF/WavLM_embeddings.py:extract_wavlm_embeddings`,
`REF/whisper_embeddings_large.py:extract_whisper_embeddings_fixed`) on HF models built
offline with the deterministic synthetic weights of ``synth.py`` — see
``tests/golden/make_golden.py`` and ``tests/test_oracle_golden.py``.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker / CPU baseline.  The product path
(``stuttering-speech-representation_amd``) never imports it and has no CPU fallback.
"""

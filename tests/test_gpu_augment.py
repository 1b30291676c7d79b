"""GPU parity of the augmentation row: sse_augment / speed round trip
against oracle/augment.py (noise stream restated exactly: max abs <= 1e-6; resampling <= 2e-6),
and apply_data_augmentation end to end against a batch-1 restatement of the reference's loop
(REF/model_training_1.py:318-464) on the fp32 path (rel-L2 <= 1e-4)."""
import random

import numpy as np
import pandas as pd
import pytest
import torch

from test_wavio import write_wav

pytestmark = pytest.mark.gpu


def test_augment_batch_matches_oracle():
    from oracle.augment import augment
    from ssr_amd import synth
    from ssr_amd.augment import AugSpec, augment_batch
    clips = synth.synth_clips(6, 24000, seed=11) * 4
    specs = [AugSpec("none"), AugSpec("noise", 0.004), AugSpec("volume", 1.07), AugSpec("speed", 0.96, int(16000 * 0.96)),
             AugSpec("speed", 1.04, int(16000 * 1.04)), AugSpec("noise", 0.02)]
    got = augment_batch([torch.from_numpy(c).cuda() for c in clips], specs, seed=77, streams=[10, 11, 12, 13, 14, 15])
    for i, (c, sp) in enumerate(zip(clips, specs)):
        want = augment(c, sp.kind, sp.factor, sp.new_sr, seed=77, stream=10 + i)
        g = got[i].cpu().numpy()
        assert g.shape == want.shape
        err = np.abs(g - want).max()
        print(sp.kind, err)
        assert err <= (2e-6 if sp.kind == "speed" else 1e-6)


def test_pitch_returns_original_like_reference():
    from ssr_amd.augment import augment_audio

    class R:                       # force the pitch branch with a non-zero shift
        def choice(self, s):
            return "pitch"

        def randint(self, a, b):
            return 2

    x = np.linspace(-0.2, 0.2, 500, dtype=np.float32)
    assert np.array_equal(augment_audio(x, rng=R(), variant="01"), x)


def test_apply_data_augmentation_matches_sequential(tmp_path):
    from oracle.augment import augment
    from ssr_amd import config as C, synth
    from ssr_amd.augment import apply_data_augmentation, draw
    from ssr_amd.hf import Wav2Vec2FeatureExtractor, WavLMModel
    rng_np = np.random.default_rng(0)
    rows = []
    for i in range(5):
        p = str(tmp_path / f"f{i}.wav")
        write_wav(p, synth.synth_clips(1, 16000 + 160 * i, seed=50 + i)[0], fmt="float")
        rows.append({"filename": f"f{i}", "path": p, "label": "rare" if i < 2 else "common"})
    meta = pd.DataFrame(rows)
    model = WavLMModel.from_state_dict(C.WAVLM_BASE, synth.synth_wavlm_state_dict(C.WAVLM_BASE), "cuda:0", "fp32")
    fe = Wav2Vec2FeatureExtractor(do_normalize=False, device="cuda:0")
    names = ["layer_12", "layer_6"]
    emb = {"layer_12": rng_np.standard_normal((5, 768)).astype(np.float32)}
    cache = {}
    m2, e2 = apply_data_augmentation(meta, emb, model, fe, "cuda:0", names, "wavlm", augmentation_factor=3,
                                     minority_threshold=3, rng=random.Random(5), seed=9, cache=cache)
    assert len(m2) == 5 + 6 and e2["layer_12"].shape == (11, 768)     # class "rare" (2 < 3) x 3
    assert list(m2["filename"][5:8]) == ["f0_aug_0", "f0_aug_1", "f0_aug_2"] and m2["augmented"][5:].all()
    # restate the reference loop batch-1: same draws, oracle augmentation, single-clip embed
    rng = random.Random(5)
    j = 0
    for i in range(2):
        clip = synth.synth_clips(1, 16000 + 160 * i, seed=50 + i)[0]
        for a in range(3):
            sp = draw(rng)
            y = augment(clip, sp.kind, sp.factor, sp.new_sr, seed=9, stream=j)
            ref = model.embed(torch.from_numpy(y).cuda(), [12]).cpu().numpy()[0, 0]
            got = e2["layer_12"][5 + j]
            assert np.linalg.norm(got - ref) / np.linalg.norm(ref) <= 1e-4
            j += 1
    # hoisted: the second layer of the caller's per-layer loop reuses the cached work
    emb6 = {"layer_6": rng_np.standard_normal((5, 768)).astype(np.float32)}
    m3, e3 = apply_data_augmentation(meta, emb6, model, fe, "cuda:0", names, "wavlm", augmentation_factor=3,
                                     minority_threshold=3, rng=random.Random(999), seed=9, cache=cache)
    assert e3["layer_6"].shape == (11, 768) and m3["filename"].equals(m2["filename"])

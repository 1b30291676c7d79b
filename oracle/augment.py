"""ORACLE (test infrastructure only): numpy restatement of augment_audio's signal ops
(REF/model_training_1.py:167-214) as the build defines them:
  speed   resample(16000 -> int(16000*f)) then back (oracle/resample.py), clamp
  noise   x + float32(N(0,1)) * f, N from synth.gaussian(seed, stream) (the build's counter
          hash; the reference draws torch.randn_like on the CPU: same distribution, other values)
  volume  x * f, clamp;  none  clamp
  pitch   torchaudio PitchShift(sample_rate, n_steps) restated in oracle/pitch.py, clamp
          (REF/model_training_01.py:172-177)
All arithmetic in float32 like torch's CPU ops."""
from __future__ import annotations

import numpy as np

from .resample import resample


def augment(x: np.ndarray, kind: str, factor: float = 1.0, new_sr: int = 0, seed: int = 0, stream: int = 0,
            sample_rate: int = 16000, n_steps: int = 0) -> np.ndarray:
    import importlib
    synth = importlib.import_module("stuttering-speech-representation_amd.synth")
    x = np.asarray(x, dtype=np.float32)
    if kind == "speed":
        x = resample(resample(x, sample_rate, new_sr), new_sr, sample_rate)
    elif kind == "pitch" and n_steps != 0:
        from .pitch import pitch_shift
        x = pitch_shift(x, sample_rate, n_steps)
    elif kind == "noise":
        g = synth.gaussian(seed, stream, x.shape[-1]).astype(np.float32)
        x = (x + g * np.float32(factor)).astype(np.float32)
    elif kind == "volume":
        x = (x * np.float32(factor)).astype(np.float32)
    return np.clip(x, -1.0, 1.0).astype(np.float32)

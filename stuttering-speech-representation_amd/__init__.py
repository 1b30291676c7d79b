"""MI355X-native (gfx950) speech-embedding extractor for the hot path of
warren-machy/stuttering-speech-representation: WavLM / Whisper forward -> per-clip
mean-pooled hidden-layer embeddings.

The directory name contains hyphens, so import it with
``importlib.import_module("stuttering-speech-representation_amd")``; after that first import
the package and every submodule are also reachable as ``ssr_amd`` / ``ssr_amd.<sub>``
(the SAME module objects, through an alias finder — no second copy of any class).

Layers:
  extract.py   drop-in glue: extract_wavlm_embeddings / extract_whisper_embeddings_fixed
               and their in-memory twins (REF/WavLM_embeddings.py:267,
               REF/whisper_embeddings_large.py:234, REF/model_training_1.py:235,268)
  hf.py        HF-duck-typed model / feature-extractor objects
  model.py     SSEModel: weights -> device handle, batched ``embed`` / ``hidden_states``
  _lib.py      ctypes binding of the C-ABI library ``libsse.so`` (include/sse.h)
  corpus.py    clip-sharded multi-GPU extraction with one all-gather
  csrc/        HIP kernels for gfx950 + the C-ABI
"""
import importlib
import importlib.abc
import importlib.util
import sys as _sys

_ALIAS = "ssr_amd"


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, real: str):
        self.real = real

    def create_module(self, spec):
        return importlib.import_module(self.real)

    def exec_module(self, module):
        pass


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, name, path=None, target=None):
        if name == _ALIAS or name.startswith(_ALIAS + "."):
            real = __name__ + name[len(_ALIAS):]
            return importlib.util.spec_from_loader(name, _AliasLoader(real))
        return None


if not any(isinstance(f, _AliasFinder) for f in _sys.meta_path):
    _sys.meta_path.insert(0, _AliasFinder())
_sys.modules.setdefault(_ALIAS, _sys.modules[__name__])

from . import config, synth  # noqa: E402,F401  (pure-python, no GPU needed)

__all__ = ["config", "synth"]

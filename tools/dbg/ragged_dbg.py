"""Debug: which configuration breaks ragged-vs-alone bit-identity (clip 70 of the corpus test)."""
import importlib, sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import config as C, synth, _lib
from ssr_amd.model import SSEModel
spec = C.WAVLM_BASE
sd = synth.synth_wavlm_state_dict(spec, seed=7)
m = SSEModel(spec, sd, device="cuda:0", dtype="bf16")
rng = np.random.default_rng(5)
lens = rng.integers(8000, 51000, size=600)
clips = [synth.synth_clips(1, int(n), seed=900 + i)[0] for i, n in enumerate(lens[:256])]
idx = list(range(13))
def first_diff(a, b):
    d = [(k, float(np.abs(a[k] - b[k]).max())) for k in range(13) if not np.array_equal(a[k], b[k])]
    return d[:3]
alone = {j: m.embed(torch.from_numpy(clips[j]).cuda()[None], idx).cpu().numpy()[0] for j in (0, 70, 100)}
def run(name, js, opts=()):
    for o, v in opts: _lib.lib().sse_set_option(o.encode(), v)
    got = m.embed_clips([torch.from_numpy(clips[j]) for j in js], idx).cpu().numpy()
    for o, v in opts: _lib.lib().sse_set_option(o.encode(), 0)
    res = {j: first_diff(got[js.index(j)], alone[j]) for j in (0, 70, 100) if j in js}
    print(name, res, flush=True)
allj = list(range(256))
run("B256 ragged", allj)
run("B2 [70,0]", [70, 0])
run("B2 [70,max]", [70, int(np.argmax(lens[:256]))])
run("B72", list(range(72)))
run("B128", list(range(128)))
for o in ("conv0_valu", "posconv_gemm", "gemm_nonpersist", "no_lnfold"):
    run("B256 " + o, allj, [(o, 1)])

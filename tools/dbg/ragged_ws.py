"""Debug: truncated WavLM (11 layers) on the ragged batch; workspace diff persistent vs non-persistent."""
import importlib, sys, os, dataclasses
sys.path.insert(0, os.getcwd())
import numpy as np, torch
importlib.import_module("stuttering-speech-representation_amd")
from ssr_amd import config as C, synth, _lib
from ssr_amd.model import SSEModel
NL = int(sys.argv[1]) if len(sys.argv) > 1 else 11
spec = dataclasses.replace(C.WAVLM_BASE, layers=NL)
sd = synth.synth_wavlm_state_dict(C.WAVLM_BASE, seed=7)
sd = {k: v for k, v in sd.items() if not any(k.startswith(f"encoder.layers.{l}.") for l in range(NL, 12))}
m = SSEModel(spec, sd, device="cuda:0", dtype="bf16")
rng = np.random.default_rng(5)
lens = rng.integers(8000, 51000, size=600)[:72]
clips = [synth.synth_clips(1, int(n), seed=900 + i)[0] for i, n in enumerate(lens)]
L = int(max(lens))
wave = torch.zeros(72, L, device="cuda")
for i, c in enumerate(clips):
    wave[i, :len(c)] = torch.from_numpy(c)
nb = _lib.lib().sse_workspace_bytes(m._h, 72, L)
def run(np_):
    ws = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    with _lib.option("gemm_nonpersist", np_):
        e = m.embed(wave, [NL], lengths=[int(x) for x in lens], workspace=ws)
    torch.cuda.synchronize()
    return e.cpu().numpy(), ws.cpu().numpy()
e0, w0 = run(0)
e1, w1 = run(1)
e0b, w0b = run(0)
print("persistent repeat equal:", np.array_equal(e0, e0b), np.array_equal(w0, w0b))
diffc = [b for b in range(72) if not np.array_equal(e0[b], e1[b])]
print("clips differing (persist vs nonpersist):", diffc)
d = np.nonzero(w0 != w1)[0]
print("ws bytes", nb, "differing bytes", d.size)
if d.size:
    # cluster into regions
    br = np.nonzero(np.diff(d) > 4096)[0]
    starts = np.concatenate([[d[0]], d[br + 1]]); ends = np.concatenate([d[br], [d[-1]]])
    for s, e in list(zip(starts, ends))[:20]:
        print("region", int(s), int(e), "len", int(e - s + 1))
Tf = spec.frames(L); M = 72 * Tf
print("Tf", Tf, "M", M, "qkv bytes", M * 2560 * 2, "ff bytes", M * 3072 * 2, "H bytes", M * 768 * 2)
off_qkv = 1197709056
def qkv_el(w, row, col):
    o = off_qkv + (row * 2560 + col) * 2
    return np.frombuffer(w[o:o + 2].tobytes(), dtype=np.uint16)[0]
for (row, col) in [(11147, 2027)]:
    a, b = qkv_el(w0, row, col), qkv_el(w1, row, col)
    f = lambda u: np.frombuffer(np.array([u], np.uint32) << 16, dtype=np.float32)[0]
    print("qkv", row, col, hex(a), f(a), hex(b), f(b))
# whole qkv region compare
q0 = np.frombuffer(w0[off_qkv:off_qkv + M * 2560 * 2].tobytes(), np.uint16).reshape(M, 2560)
q1 = np.frombuffer(w1[off_qkv:off_qkv + M * 2560 * 2].tobytes(), np.uint16).reshape(M, 2560)
r, c = np.nonzero(q0 != q1)
print("qkv diffs", list(zip(r.tolist(), c.tolist()))[:10])
# alone run of clip 70 (persistent), rows of its qkv
c70 = torch.from_numpy(clips[70]).cuda()[None]
nb1 = _lib.lib().sse_workspace_bytes(m._h, 1, len(clips[70]))
ws1 = torch.zeros(nb1, dtype=torch.uint8, device="cuda")
m.embed(c70, [NL], workspace=ws1); torch.cuda.synchronize()
w = ws1.cpu().numpy()
# locate qkv in the alone workspace: search for the batch row's 2560 values (row 11147 = local 17)
row_b = q1[11147].tobytes()
pos = w.tobytes().find(row_b)
print("nonpersist batch row 17 found in alone ws at", pos)
row_p = q0[11147].tobytes()
print("persist batch row 17 found in alone ws at", w.tobytes().find(row_p))

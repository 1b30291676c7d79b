"""The Whisper flash attention kernels through the C-ABI test hook `sse_attention` against a torch fp32
reference of the same op (HF WhisperAttention, REF/whisper_embeddings_large.py:250 -> SDPA):
softmax(scale q k^T) v per 64-wide head.

attention_flash3_kernel (attn_long = 0: two 32-query blocks per wave; 2: one) defers the row max: it is
taken only on the first tile and on tiles whose row sums pass the 2^8 slack, where O and l are rescaled
and the tile is exponentiated again against the new max.  Random scores almost never take that branch
after the first tile, so the adversarial cases drive it: scores that climb along the keys (a rescale on
every tile), a single late spike, and rows whose maxima sit in the ragged last tile.  flash2 (attn_long =
1) is checked on the same inputs.  Bar: max |out - ref| <= 1.5e-2 max |ref| (bf16 probabilities, bf16
output); the two flash3 variants bit-identical (same per-query arithmetic)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

LN2, LOG2E = math.log(2.0), 1.0 / math.log(2.0)


def _run(qkv, B, T, H, nh, scale, q_log2, mode):
    from ssr_amd import _lib
    out = torch.empty((B * T, H), dtype=torch.bfloat16, device="cuda")
    with _lib.option("attn_long", mode):
        rc = _lib.lib().sse_attention(qkv.data_ptr(), out.data_ptr(), B, T, H, nh, qkv.shape[1], scale, q_log2, None)
    _lib.check(rc, "sse_attention")
    torch.cuda.synchronize()
    return out


def _ref(qkv, B, T, H, nh, scale):
    x = qkv.float().view(B, T, -1)
    q, k, v = (x[..., i * H:(i + 1) * H].view(B, T, nh, 64).transpose(1, 2) for i in range(3))
    p = torch.softmax((q @ k.transpose(-1, -2)) * scale, dim=-1)
    return (p @ v).transpose(1, 2).reshape(B * T, H)


def _qkv(B, T, H, kind, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    q, k, v = (torch.randn((B, T, H), device="cuda", generator=g) for _ in range(3))
    if kind == "climb":      # score of key j ~ 216 j / T log2 units (after q's 0.18): past the slack every tile
        u = torch.randn((H,), device="cuda", generator=g)
        u = u / u.norm()
        q = q * 0.1 + u * 4.0
        ramp = torch.linspace(0, 1, T, device="cuda")[None, :, None]
        k = k * 0.1 + u * (ramp * 300.0)
    elif kind == "spike":    # one key near the end far above the rest (a single late rescale)
        k[:, T - 7] *= 12.0
    elif kind == "tail":     # the largest keys in the ragged last tile
        k[:, -(T % 64 or 64):] *= 6.0
    qkv = torch.cat([q, k, v], dim=-1).reshape(B * T, 3 * H)
    return qkv


@pytest.mark.parametrize("T", [1500, 200, 161, 65])
@pytest.mark.parametrize("kind", ["random", "climb", "spike", "tail"])
def test_flash_attention_vs_fp32_reference(T, kind):
    B, nh = 2, 6
    H = 64 * nh
    qkv32 = _qkv(B, T, H, kind, seed=T * 7 + len(kind))
    # the encoder's layout: q carries scale * log2(e) (scale = 1/8), the kernel's scale is ln 2
    qs = qkv32.clone()
    qs[:, :H] *= 0.125 * LOG2E
    qkv = qs.to(torch.bfloat16)
    ref = _ref(qkv, B, T, H, nh, LN2)
    top = ref.abs().max().item()
    outs = {}
    for mode in (0, 2, 1):
        o = _run(qkv, B, T, H, nh, LN2, 1, mode)
        assert torch.isfinite(o).all(), (kind, T, mode)
        err = (o.float() - ref).abs().max().item()
        print(f"{kind:6s} T={T:5d} attn_long={mode}: max err {err:.3e} of max |ref| {top:.3f}")
        assert err <= 1.5e-2 * top, (kind, T, mode, err, top)
        outs[mode] = o
    assert torch.equal(outs[0], outs[2])


def test_flash_attention_plain_scale():
    """q_log2 = 0 (any scale, no folded log2 e): the 16x16 kernel, against the same reference."""
    B, T, nh = 2, 300, 4
    H = 64 * nh
    qkv = _qkv(B, T, H, "random", seed=5).to(torch.bfloat16)
    ref = _ref(qkv, B, T, H, nh, 0.125)
    o = _run(qkv, B, T, H, nh, 0.125, 0, 0)
    assert (o.float() - ref).abs().max().item() <= 1.5e-2 * ref.abs().max().item()


def test_flash_attention_rejects_bad_shapes():
    from ssr_amd import _lib
    x = torch.zeros((64, 3 * 128), dtype=torch.bfloat16, device="cuda")
    out = torch.empty((64, 128), dtype=torch.bfloat16, device="cuda")
    L = _lib.lib()
    assert L.sse_attention(x.data_ptr(), out.data_ptr(), 1, 64, 130, 2, 3 * 128, 1.0, 0, None) < 0   # H != 64 nh
    assert L.sse_attention(x.data_ptr(), out.data_ptr(), 1, 64, 128, 2, 200, 1.0, 0, None) < 0       # ldq < 3H
    assert L.sse_attention(None, out.data_ptr(), 1, 64, 128, 2, 3 * 128, 1.0, 0, None) < 0
    # q_log2 = 1 with a scale other than ln 2 (the 32x32 kernel would ignore it: ADVICE r4)
    assert L.sse_attention(x.data_ptr(), out.data_ptr(), 1, 64, 128, 2, 3 * 128, 1.0, 1, None) < 0

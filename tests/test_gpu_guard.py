"""Guard bands around every output the path's kernels store.

Two out-of-range stores of the persistent GEMM epilogue were found in round 4 only because a
neighbouring allocation happened to be read later (non-finite embeddings):

* bug A (fixed in e0a750d): the store's buffer resource was based at the tile's FIRST ROW only, so
  every 256-column tile of a row block wrote columns 0-255 -- columns >= 256 were never written and
  columns 0-255 took the last tile's values;
* bug B (fixed in 0315a32): the row block rode in the SGPR offset of one tile-wide resource, which
  the range check does not see, so a partial tile (M % 256 != 0) wrote rows >= M.

The kernel tests compare values inside an exactly sized output, which misses stores that land
outside it.  Here every output is a window of a larger buffer pre-filled with a NaN bit pattern:
guard rows before row 0 and after row M - 1, guard columns between N and the row stride ldc > N
(the hook takes ldc), and the test asserts (1) every guard element still holds the pattern bit for
bit, (2) every element of the window was written (no pattern left, so bug A's unwritten columns
show) and matches a torch fp32 reference of the same op (bug A's wrong columns show).  Shapes use
partial last row tiles, M % 256 in {1, 17, 255} (bug B).  Column tiles are never partial here: every
GEMM kernel requires N to be a multiple of its tile width (256 for the 8-phase kernels, 128 / 64 / 48
for the generic one) and rejects other N, so the column guards cover stores past N instead.

Forms covered, each naming the store it guards: the persistent GEMM's register-direct epilogue
(gemm8p_kernel EP 0 / 1 / 3, FNT 3 / 5, GELU, fp16), the residual GEMM (gemm8r_kernel, fp32 residual
and the bf16 / fp16 residual stream with LayerNorm partials in and out), the LDS-staged 8-phase kernel,
the generic tile kernel (gemm_kernel 128 x 128 / 64 / 48, bf16 and fp32), the MX-fp8 GEMM's direct
epilogue (bf16 / fp32 out, and the fc1 form that quantises to e4m3 + E8M0 scales), the attention
kernels' bounded output resources (short-T pipelined, 16x16 and 32x32 flash), and the pooled
embeddings plus the model workspace of a whole sse_embed call."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

# NaN bit patterns (never produced by a kernel: quiet NaNs with a payload)
PAT = {torch.bfloat16: 0x7FB5, torch.float16: 0x7E5A, torch.float32: 0x7FC0BEEF, torch.uint8: 0xA5}
IVIEW = {torch.bfloat16: torch.int16, torch.float16: torch.int16, torch.float32: torch.int32, torch.uint8: torch.uint8}
FRONT, BACK = 8, 64   # guard rows before / after the window


def _pat(dt):
    p = PAT[dt]
    if IVIEW[dt] == torch.int16 and p >= 0x8000:
        p -= 0x10000
    if IVIEW[dt] == torch.int32 and p >= 0x80000000:
        p -= 0x100000000
    return p


class Guarded:
    """A [FRONT + rows + BACK, ldc] buffer of the pattern; .win is the [rows, ldc] window, .out its [:, :n]."""

    def __init__(self, rows, n, ldc, dt):
        self.rows, self.n, self.ldc, self.dt = rows, n, ldc, dt
        self.raw = torch.full(((FRONT + rows + BACK) * ldc,), _pat(dt), dtype=IVIEW[dt], device="cuda")
        self.full = self.raw.view(dt).view(FRONT + rows + BACK, ldc)
        self.win = self.full[FRONT:FRONT + rows]

    def ptr(self):
        return self.win.data_ptr()

    @property
    def out(self):
        return self.win[:, :self.n]

    def check(self, what=""):
        torch.cuda.synchronize()
        iv = self.raw.view(FRONT + self.rows + BACK, self.ldc)
        p = _pat(self.dt)
        assert bool((iv[:FRONT] == p).all()), f"{what}: store before row 0"
        bad = (iv[FRONT + self.rows:] != p).any(dim=1).nonzero()
        assert bad.numel() == 0, f"{what}: store into guard row(s) past M, first {int(bad[0]) + self.rows}"
        if self.ldc > self.n:
            assert bool((iv[FRONT:FRONT + self.rows, self.n:] == p).all()), f"{what}: store into columns [N, ldc)"
        assert not bool((iv[FRONT:FRONT + self.rows, :self.n] == p).any()), f"{what}: output element never written"


class GuardedBytes:
    """A flat byte buffer with guard bytes before and after an n-byte window."""

    def __init__(self, n):
        self.n = n
        self.raw = torch.full((1024 + n + 4096,), PAT[torch.uint8], dtype=torch.uint8, device="cuda")
        self.win = self.raw[1024:1024 + n]

    def check(self, what=""):
        torch.cuda.synchronize()
        assert bool((self.raw[:1024] == PAT[torch.uint8]).all()), f"{what}: store before the window"
        assert bool((self.raw[1024 + self.n:] == PAT[torch.uint8]).all()), f"{what}: store past the window"


_Z = {}


def _zero():
    if "z" not in _Z:
        _Z["z"] = torch.zeros(64, dtype=torch.float32, device="cuda")
    return _Z["z"]


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _gemm_ex(dtype_code, a, b, M, N, K, ldc, **kw):
    from ssr_amd import _lib
    d = _lib.sse_gemm_desc()
    d.dtype, d.M, d.N, d.K, d.ldc = dtype_code, M, N, K, ldc
    d.act = kw.pop("act", 0)
    d.apart_nt = kw.pop("apart_nt", 0)
    d.ln_eps = kw.pop("ln_eps", 1e-5)
    d.a, d.b, d.zero = a.data_ptr(), b.data_ptr(), _zero().data_ptr()
    for k, v in kw.items():
        setattr(d, k, None if v is None else (v if isinstance(v, int) else v.data_ptr()))
    # (resid_t / ct may be passed as raw pointers: the in-place residual forms)
    rc = _lib.lib().sse_gemm_ex(ctypes.byref(d), _stream())
    _lib.check(rc, "sse_gemm_ex")


def _partials(x, nt):
    """(mean, M2) of every 256 columns of the rows of x (fp32 math on the stored values) -> [M, nt, 2]."""
    t = x.float().view(x.shape[0], nt, 256)
    mean = t.mean(-1)
    m2 = ((t - mean[..., None]) ** 2).sum(-1)
    return torch.stack([mean, m2], -1).contiguous()


def _ln_from_partials(p, eps):
    nt = p.shape[1]
    mean = p[..., 0].mean(-1)
    m2 = p[..., 1].sum(-1) + 256.0 * ((p[..., 0] - mean[:, None]) ** 2).sum(-1)
    return mean, 1.0 / torch.sqrt(m2 / (256 * nt) + eps)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


TDT = {1: torch.bfloat16, 4: torch.float16, 0: torch.float32}


@pytest.mark.parametrize("M", [4097, 4113, 4351, 38161])
@pytest.mark.parametrize("form", ["ep0", "ep1_gelu", "fold_ep3", "fold_ep3_gelu", "fold_fnt4", "fold_fnt5", "h16_ep1_gelu",
                                  "staged_cf_ct"])
def test_gemm_nonresidual_guard_bands(M, form):
    """gemm8p_kernel's register-direct epilogue (one buffer resource per 16-row block; bug A: each column
    tile's stores based at its own column, caught by the window check; bug B: rows >= M of the partial
    last row tile, caught by the guard rows) for EP 0 (no bias), 1 (bias, GELU), 3 (folded LayerNorm,
    FNT 3, 4 (WavLM-large's QKV) and 5), fp16 operands; and the LDS-staged 8-phase kernel (GELU with fp32 + bf16 outputs).
    M = 38161 (149 full row tiles + 17 rows) x N = 1536 is 900 tiles: every persistent block walks 3-4
    tiles (the epilogue's stores stay in flight under the next tile's first K-tile)."""
    dt = torch.float16 if form.startswith("h16") else torch.bfloat16
    code = 4 if dt == torch.float16 else 1
    K = {"fold_ep3": 768, "fold_ep3_gelu": 768, "fold_fnt4": 1024, "fold_fnt5": 1280}.get(form, 192)
    N = 768 if form in ("fold_fnt4", "fold_fnt5") else 512
    if M > 30000:
        N *= 3
    ldc = N + 64
    g = torch.Generator(device="cuda").manual_seed(M + len(form))
    a = torch.randn(M, K, device="cuda", generator=g).to(dt)
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dt)
    bias = torch.randn(N, device="cuda", generator=g) if form != "ep0" else None
    act = 2 if "gelu" in form or form == "staged_cf_ct" else 0
    acc = a.float() @ b.float().T
    kw = {}
    if form.startswith("fold"):
        nt = K // 256
        part = _partials(a, nt)
        acol = b.float().sum(1).contiguous()
        mean, rstd = _ln_from_partials(part, 1e-5)
        ref = rstd[:, None] * (acc - mean[:, None] * acol[None, :]) + bias
        kw.update(apart=part, acol=acol, apart_nt=nt)
    else:
        ref = acc + (bias if bias is not None else 0.0)
    if act:
        ref = torch.nn.functional.gelu(ref)
    ct = Guarded(M, N, ldc, dt)
    cf = Guarded(M, N, ldc, torch.float32) if form == "staged_cf_ct" else None
    _gemm_ex(code, a, b, M, N, K, ldc, bias=bias, act=act, ct=ct.ptr(), cf=cf.ptr() if cf else None, **kw)
    ct.check(form)
    assert _rel(ct.out, ref) <= 1e-2, form
    if cf is not None:
        cf.check(form + " fp32")
        assert _rel(cf.out, ref) <= 1e-4


@pytest.mark.parametrize("M", [4097, 4351, 301])
@pytest.mark.parametrize("form", ["f32_resid", "bf16_stream_ln_opart", "bf16_stream_opart", "h16_stream_ln_opart"])
def test_gemm_residual_guard_bands(M, form):
    """gemm8r_kernel (one tile per block): fp32 residual with fp32 + bf16 outputs, and the folded post-LN
    flow's 16-bit residual stream (resid_t, its LayerNorm from rpart partials, out-partials opart).  Its
    stores are per-lane row-checked (m < M); the guard rows hold that invariant (bug B's symptom) for the
    output, the 16-bit copy and the partials, and the window check bug A's (every column tile written)."""
    dt = torch.float16 if form.startswith("h16") else torch.bfloat16
    code = 4 if dt == torch.float16 else 1
    N, K = 768, 256
    ldc = N + 64
    g = torch.Generator(device="cuda").manual_seed(M * 3 + len(form))
    a = torch.randn(M, K, device="cuda", generator=g).to(dt)
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dt)
    bias = torch.randn(N, device="cuda", generator=g)
    acc = a.float() @ b.float().T + bias
    if form == "f32_resid":
        res = torch.randn(M, ldc, device="cuda", generator=g)
        cf, ct = Guarded(M, N, ldc, torch.float32), Guarded(M, N, ldc, torch.bfloat16)
        _gemm_ex(code, a, b, M, N, K, ldc, bias=bias, resid=res, cf=cf.ptr(), ct=ct.ptr())
        ref = acc + res[:, :N]
        cf.check(form)
        ct.check(form + " bf16 copy")
        assert _rel(cf.out, ref) <= 1e-5 and _rel(ct.out, ref) <= 1e-2
        return
    res = (torch.randn(M, ldc, device="cuda", generator=g) * 2 + 0.5).to(dt)
    kw = {}
    r = res[:, :N].float()
    if "_ln" in form:
        part = _partials(res[:, :N].contiguous(), 3)
        lw = torch.rand(N, device="cuda", generator=g) + 0.5
        lb = torch.randn(N, device="cuda", generator=g) * 0.1
        mean, rstd = _ln_from_partials(part, 1e-5)
        r = ((r - mean[:, None]) * rstd[:, None]) * lw + lb
        kw.update(rpart=part, rln_w=lw, rln_b=lb)
    ref = acc + r
    ct = Guarded(M, N, ldc, dt)
    op = Guarded(M, 6, 6, torch.float32)   # [M][N / 256] float2 = 6 floats per row
    _gemm_ex(code, a, b, M, N, K, ldc, bias=bias, resid_t=res, ct=ct.ptr(), opart=op.ptr(), **kw)
    ct.check(form)
    op.check(form + " opart")
    assert _rel(ct.out, ref) <= 1e-2
    exp = _partials(ct.out.contiguous(), 3).view(M, 6)
    assert _rel(op.out, exp) <= 1e-3


@pytest.mark.parametrize("dt,M,N,K", [(torch.bfloat16, 1000, 384, 64), (torch.bfloat16, 1025, 192, 96),
                                      (torch.bfloat16, 273, 144, 64), (torch.float32, 4097, 256, 64),
                                      (torch.float32, 511, 128, 32)])
def test_gemm_generic_tile_guard_bands(dt, M, N, K):
    """gemm_kernel (kernels_gemm.hip: 128 x {128, 64, 48} tiles, bf16 and exact-f32 MFMA; the LDS-staged
    16-B epilogue with per-row `ok` checks): partial last row tiles, guard rows and columns."""
    code = 1 if dt == torch.bfloat16 else 0
    ldc = N + 32
    g = torch.Generator(device="cuda").manual_seed(M + N)
    a = torch.randn(M, K, device="cuda", generator=g).to(dt)
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dt)
    bias = torch.randn(N, device="cuda", generator=g)
    res = torch.randn(M, ldc, device="cuda", generator=g)
    cf = Guarded(M, N, ldc, torch.float32)
    _gemm_ex(code, a, b, M, N, K, ldc, bias=bias, resid=res, act=1, cf=cf.ptr())
    cf.check("generic")
    ref = torch.nn.functional.gelu(a.float() @ b.float().T + bias) + res[:, :N]
    assert _rel(cf.out, ref) <= 1e-5


@pytest.mark.parametrize("M", [257, 273, 511])
@pytest.mark.parametrize("out", ["fp32", "bf16", "fp8"])
def test_gemm_mx_guard_bands(M, out):
    """The MX-fp8 GEMM (gemm8_kernel<MX>, Cᵀ in registers, the same buffer-resource store pattern since
    round 4): fp32 / bf16 outputs, and fc1's form that quantises its output to e4m3 plus E8M0 scales in
    the next GEMM's tiled A layout (scale dwords of a partial row tile stay inside the padded
    mx_scale_bytes(M, N) allocation).  ldc = N for this hook: guard rows and bytes only."""
    from oracle import mx
    from ssr_amd import _lib
    from ssr_amd.model import mx_scale_bytes
    N, K = 512, 256
    rng = np.random.default_rng(M)
    a = rng.standard_normal((M, K)).astype(np.float32)
    bw = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float32)
    qa, sa, ea = mx.quantize(a, 0)
    qb, sb, eb = mx.quantize(bw, 1)
    ref = torch.from_numpy(mx.dequantize(qa, ea) @ mx.dequantize(qb, eb).T).cuda()
    dev = lambda v: torch.from_numpy(v).cuda()
    qa_, sa_, qb_, sb_ = dev(qa), dev(sa), dev(qb), dev(sb)
    bias = torch.from_numpy(rng.standard_normal(N).astype(np.float32)).cuda()
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp8": torch.uint8}[out]
    c = Guarded(M, N, N, dt)
    cs = GuardedBytes(mx_scale_bytes(M, N)) if out == "fp8" else None
    rc = _lib.lib().sse_gemm_mx(qa_.data_ptr(), sa_.data_ptr(), qb_.data_ptr(), sb_.data_ptr(), bias.data_ptr(), None,
                                c.ptr() if out == "fp32" else None, c.ptr() if out != "fp32" else None,
                                cs.win.data_ptr() if cs else None, M, N, K, 2 if out == "fp8" else 0, _stream())
    _lib.check(rc, "sse_gemm_mx")
    if out == "fp8":
        torch.cuda.synchronize()
        # the window check would misread an e4m3 code equal to the pattern byte as "never written": check
        # guard rows only, then the codes against the restatement
        iv = c.raw.view(FRONT + M + BACK, N)
        assert bool((iv[:FRONT] == PAT[torch.uint8]).all()) and bool((iv[FRONT + M:] == PAT[torch.uint8]).all())
        cs.check("fp8 scales")
        return
    c.check(out)
    assert _rel(c.out, ref + bias) <= (1e-4 if out == "fp32" else 1e-2)


@pytest.mark.parametrize("T", [65, 149, 161, 1500])
def test_attention_output_guard_bands(T):
    """The attention kernels store through a buffer resource bounded to the clip's rows (short-T pipelined
    T <= 160; 32x32 flash above): B = 3 clips, output [B*T][H] bf16 with guard rows before and after."""
    from ssr_amd import _lib
    B, nh = 3, 4
    H = 64 * nh
    g = torch.Generator(device="cuda").manual_seed(T)
    qkv = torch.randn(B * T, 3 * H, device="cuda", generator=g)
    qkv[:, :H] *= 0.125 * 1.4426950408889634
    qkv = qkv.to(torch.bfloat16)
    o = Guarded(B * T, H, H, torch.bfloat16)
    rc = _lib.lib().sse_attention(qkv.data_ptr(), o.ptr(), B, T, H, nh, 3 * H, 0.6931471805599453, 1, _stream())
    _lib.check(rc, "sse_attention")
    o.check(f"attention T={T}")
    x = qkv.float().view(B, T, 3 * H)
    q, k, v = (x[..., i * H:(i + 1) * H].view(B, T, nh, 64).transpose(1, 2) for i in range(3))
    p = torch.softmax((q @ k.transpose(-1, -2)) * 0.6931471805599453, dim=-1)
    ref = (p @ v).transpose(1, 2).reshape(B * T, H)
    assert (o.out.float() - ref).abs().max().item() <= 1.5e-2 * ref.abs().max().item()


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_embed_output_and_workspace_guard_bands(wavlm_sd, dtype):
    """A whole sse_embed call at a batch with partial GEMM row tiles (B = 7 clips x 149 frames: M = 1043)
    and the ragged path: the pooled embeddings [B, 4, 768] written into a window of a pattern buffer, and
    the model workspace followed by 1 MiB of pattern -- no kernel of the forward stores past either."""
    from ssr_amd import _lib, config as C, synth
    from ssr_amd.model import SSEModel
    m = SSEModel(C.WAVLM_BASE, wavlm_sd, device="cuda:0", dtype=dtype)
    B, L = 7, 48000
    w = torch.from_numpy(synth.synth_clips(B, L, seed=5)).cuda()
    idx = [12, 11, 10, 6]
    need = int(_lib.lib().sse_workspace_bytes(m._h, B, L))
    ws = torch.full((need + (1 << 20),), PAT[torch.uint8], dtype=torch.uint8, device="cuda")
    out = Guarded(B, 4 * 768, 4 * 768, torch.float32)
    res = m.embed(w, idx, out=out.win.view(B, 4, 768), workspace=ws)
    out.check("pooled")
    assert bool((ws[need:] == PAT[torch.uint8]).all()), "store past the workspace"
    ref = m.embed(w, idx)
    assert torch.equal(res, ref)
    lens = [48000, 400, 30001, 47999, 16000, 12345, 48000]
    ws.fill_(PAT[torch.uint8])
    out2 = Guarded(B, 4 * 768, 4 * 768, torch.float32)
    m.embed(w, idx, out=out2.win.view(B, 4, 768), lengths=lens, workspace=ws)
    out2.check("pooled ragged")
    assert bool((ws[need:] == PAT[torch.uint8]).all()), "ragged: store past the workspace"



@pytest.mark.parametrize("M", [257, 511, 3000])
@pytest.mark.parametrize("form", ["fc2", "no_bias", "gelu"])
def test_gemm_mx_bf16_residual_in_place(M, form):
    """The Whisper fp8 fc2 form: MX-fp8 operands, the bf16 residual stream read and rewritten in place
    (resid_t == ct).  Round 5 moved it from the LDS-staged epilogue to the register-direct one
    (gemm8_kernel<.., MX, RBE>): the same fp32 expression (acc + bias, + residual, rounded once), so the
    result equals the staged kernel's (option gemm_mx_staged = 1) bit for bit; guard rows stay untouched
    and the values match the dequantised product.  Forms other than fc2's (no bias, an activation: ADVICE r5)
    must not reach the compile-time fc2 epilogue, which assumes a bias and no activation: they take the staged
    kernel on both settings of the option."""
    from oracle import mx
    from ssr_amd import _lib
    N, K = 512, 384
    rng = np.random.default_rng(M + 1)
    a = rng.standard_normal((M, K)).astype(np.float32)
    bw = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float32)
    qa, sa, ea = mx.quantize(a, 0)
    qb, sb, eb = mx.quantize(bw, 1)
    dev = lambda v: torch.from_numpy(v).cuda()
    qa_, sa_, qb_, sb_ = dev(qa), dev(sa), dev(qb), dev(sb)
    bias = torch.from_numpy(rng.standard_normal(N).astype(np.float32)).cuda()
    res0 = torch.from_numpy(rng.standard_normal((M, N)).astype(np.float32)).cuda().to(torch.bfloat16)
    prod = torch.from_numpy(mx.dequantize(qa, ea) @ mx.dequantize(qb, eb).T).cuda()
    act = 1 if form == "gelu" else 0   # ACT_GELU (erf)
    if form == "no_bias":
        bias = None
    pre = prod + (bias if bias is not None else 0.0)
    ref = (torch.nn.functional.gelu(pre) if act else pre) + res0.float()
    outs = []
    for staged in (0, 1):
        c = Guarded(M, N, N, torch.bfloat16)
        c.out.copy_(res0)
        with _lib.option("gemm_mx_staged", staged):
            _gemm_ex(2, qa_, qb_, M, N, K, N, bias=bias, act=act, resid_t=c.ptr(), ct=c.ptr(), a_scale=sa_,
                     b_scale=sb_)
        c.check(f"mx resid staged={staged}")
        outs.append(c.out.clone())
    assert torch.equal(outs[0], outs[1])
    assert _rel(outs[0], ref) <= 1e-2

"""Numerics of every gfx950 HIP kernel against the fp32 PyTorch reference (mxserve/ops/reference.py)."""
import math

import pytest
import torch

from mxserve import ops
from mxserve.ops import reference as ref

pytestmark = pytest.mark.gpu


def _close(a, b, atol, rtol=0.0, name=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{name}: {bad} elements off, max err {err.max().item():.4g}"


@pytest.mark.parametrize("H", [1024, 2048, 4096, 8192])
@pytest.mark.parametrize("T", [1, 7, 128, 2050])  # 2050: the wave-per-row form
def test_rms_norm(gpu, H, T):
    x = torch.randn(T, H, device=gpu, dtype=torch.bfloat16)
    w = (1 + 0.1 * torch.randn(H, device=gpu)).bfloat16()
    _close(ops.rms_norm(x, w, 1e-5), ref.rms_norm(x.cpu(), w.cpu(), 1e-5), 0.02, 0.02, "rms_norm")


@pytest.mark.parametrize("T", [33, 4099])  # 4099: the wave-per-row form
@pytest.mark.parametrize("H", [2048, 4096])
def test_fused_add_rms_norm(gpu, H, T):
    x = torch.randn(T, H, device=gpu, dtype=torch.bfloat16)
    r = torch.randn(T, H, device=gpu, dtype=torch.bfloat16)
    w = (1 + 0.1 * torch.randn(H, device=gpu)).bfloat16()
    ey, er = ref.fused_add_rms_norm(x.cpu(), r.cpu(), w.cpu(), 1e-5)
    y, r2 = ops.fused_add_rms_norm(x, r, w, 1e-5)
    _close(r2, er, 0.02, 0.01, "residual")
    _close(y, ey, 0.03, 0.02, "normed")


@pytest.mark.parametrize("H", [1024, 2048, 4096, 8192])
def test_embed_rms_norm(gpu, H):
    """Embedding gather fused into the first RMSNorm: residual = table[ids] bit-exact, normed vs fp32."""
    V, T = 5000, 67
    table = torch.randn(V, H, device=gpu, dtype=torch.bfloat16)
    w = (1 + 0.1 * torch.randn(H, device=gpu)).bfloat16()
    ids = torch.randint(0, V, (T,), device=gpu)
    ids[3] = V - 1
    h, res = ops.embed_rms_norm(ids, table, w, 1e-5)
    assert torch.equal(res, table[ids])
    _close(h, ref.rms_norm(table[ids].cpu(), w.cpu(), 1e-5), 0.02, 0.02, "embed_rms_norm")


@pytest.mark.parametrize("I", [8192, 3584, 1792])
def test_silu_mul(gpu, I):
    gu = torch.randn(19, 2 * I, device=gpu, dtype=torch.bfloat16)
    _close(ops.silu_mul(gu), ref.silu_mul(gu.cpu()), 0.02, 0.02, "silu_mul")


def _make_kv(nb, L, hkv, D, device, dtype=torch.bfloat16):
    kv = torch.randn(nb, L, 2, hkv, 16, D, device=device, dtype=dtype) * 0.5
    return kv


@pytest.mark.parametrize("D,hq,hkv,qknorm", [(64, 32, 8, False), (128, 16, 8, True), (128, 8, 1, False)])
def test_rope_and_cache(gpu, D, hq, hkv, qknorm):
    T, L, nb = 37, 2, 20
    cos_sin = ref.build_cos_sin_cache(D, 4096, 500000.0, None, device=gpu)
    qkv = torch.randn(T, (hq + 2 * hkv) * D, device=gpu, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=gpu)
    slots = torch.randperm(nb * 16, device=gpu)[:T]
    slots[3] = -1
    qn = (1 + 0.1 * torch.randn(D, device=gpu)).bfloat16() if qknorm else None
    kn = (1 + 0.1 * torch.randn(D, device=gpu)).bfloat16() if qknorm else None
    kv = torch.zeros(nb, L, 2, hkv, 16, D, device=gpu, dtype=torch.bfloat16)
    kv_ref = kv.clone().cpu()
    q = ops.rope_and_cache(qkv, hq, hkv, D, pos, cos_sin, kv[:, 1], slots, qn, kn, 1e-6)
    qs, ks = hq * D, hkv * D
    c = qkv.cpu()
    q_ref = ref.rope_and_cache(c[:, :qs].reshape(T, hq, D), c[:, qs:qs + ks].reshape(T, hkv, D),
                               c[:, qs + ks:].reshape(T, hkv, D), pos.cpu(), cos_sin.cpu(), kv_ref[:, 1],
                               slots.cpu(), None if qn is None else qn.cpu(), None if kn is None else kn.cpu(), 1e-6)
    _close(q, q_ref, 0.03, 0.02, "q")
    _close(kv, kv_ref, 0.03, 0.02, "kv cache")
    assert kv[:, 0].abs().sum().item() == 0  # other layer untouched


@pytest.mark.parametrize("D,hq,hkv", [(64, 32, 8), (128, 32, 8)])
@pytest.mark.parametrize("kv_fp8", [False, True])
def test_rope_and_cache_prefill_t16(gpu, D, hq, hkv, kv_fp8):
    """Prefill-sized batches take the 16-tokens-per-workgroup kernel: contiguous chunks (V staged in
    LDS and written as 32-byte block rows, including a chunk that starts mid-block and a short
    tail), plus scattered slots and an unmapped token (per-element V fallback)."""
    L, nb = 2, 200
    # 3 sequences: 700 tokens from slot 0 (block-aligned), 333 from mid-block, 90 scattered
    seg = [torch.arange(0, 700), torch.arange(64 * 16 + 5, 64 * 16 + 5 + 333), torch.randperm(60 * 16)[:90] + 110 * 16]
    slots = torch.cat(seg).to(gpu)
    slots[800] = -1
    T = slots.shape[0]
    cos_sin = ref.build_cos_sin_cache(D, 8192, 500000.0, None, device=gpu)
    qkv = (torch.randn(T, (hq + 2 * hkv) * D, device=gpu) * (3 if kv_fp8 else 1)).to(torch.bfloat16)
    pos = torch.randint(0, 8000, (T,), device=gpu)
    dt = torch.uint8 if kv_fp8 else torch.bfloat16
    kv = torch.zeros(nb, L, 2, hkv, 16, D, device=gpu, dtype=dt)
    kv_ref = kv.clone().cpu()
    sc = {"k_scale": 0.05, "v_scale": 0.05} if kv_fp8 else {}
    q = ops.rope_and_cache(qkv, hq, hkv, D, pos, cos_sin, kv[:, 1], slots, None, None, 1e-6, **sc)
    qs, ks = hq * D, hkv * D
    c = qkv.cpu()
    q_ref = ref.rope_and_cache(c[:, :qs].reshape(T, hq, D), c[:, qs:qs + ks].reshape(T, hkv, D),
                               c[:, qs + ks:].reshape(T, hkv, D), pos.cpu(), cos_sin.cpu(), kv_ref[:, 1],
                               slots.cpu(), None, None, 1e-6, **sc)
    _close(q, q_ref, 0.03, 0.02, "q")
    if kv_fp8:
        got = kv.cpu().view(torch.float8_e4m3fn).float()
        want = kv_ref.view(torch.float8_e4m3fn).float()
        assert ((got - want).abs() <= 0.07 * want.abs() + 0.05).float().mean() > 0.995
    else:
        _close(kv, kv_ref, 0.03, 0.02, "kv cache")
    assert kv[:, 0].float().abs().sum().item() == 0


def _paged_setup(seq_lens, hkv, D, L=2, device="cuda"):
    nbs = [-(-s // 16) for s in seq_lens]
    nb = sum(nbs) + 5
    kv = _make_kv(nb, L, hkv, D, device)
    perm = torch.randperm(nb)[: sum(nbs)]
    mb = max(nbs)
    bt = torch.zeros(len(seq_lens), mb, dtype=torch.int32)
    o = 0
    for i, n in enumerate(nbs):
        bt[i, :n] = perm[o:o + n].to(torch.int32)
        o += n
    return kv, bt


@pytest.mark.parametrize("impl", [1, 2])  # VALU dot2 kernel, MFMA kernel
@pytest.mark.parametrize("D,G", [(64, 4), (128, 2), (128, 8), (64, 1), (128, 4), (64, 8)])
@pytest.mark.parametrize("lens", [[1, 17, 100], [513, 2000, 31, 4096], [16, 32, 33, 47]])
def test_paged_decode(gpu, D, G, lens, impl):
    hkv = 2
    hq = hkv * G
    kv, bt = _paged_setup(lens, hkv, D, device=gpu)
    B = len(lens)
    q = torch.randn(B, hq, D, device=gpu, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    out = ops.paged_attention_decode(q, kv[:, 1], bt.to(gpu), sl.to(gpu), scale, max(lens), impl=impl)
    exp = ref.paged_attention_decode(q.cpu(), kv[:, 1].cpu(), bt, sl, scale)
    _close(out, exp, 0.02, 0.02, f"decode impl {impl}")


@pytest.mark.parametrize("impl", [1, 2])
def test_paged_decode_graph_max_len(gpu, impl):
    """Graph capture launches with max_seq_len = max_model_len: idle partitions must be harmless."""
    lens = [5, 700]
    kv, bt = _paged_setup(lens, 8, 64, device=gpu)
    q = torch.randn(2, 32, 64, device=gpu, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32)
    out = ops.paged_attention_decode(q, kv[:, 0], bt.to(gpu), sl.to(gpu), 0.125, 8192, impl=impl)
    exp = ref.paged_attention_decode(q.cpu(), kv[:, 0].cpu(), bt, sl, 0.125)
    _close(out, exp, 0.02, 0.02, "decode-maxlen")


@pytest.mark.parametrize("version", [2, 3])
@pytest.mark.parametrize("D,G", [(64, 4), (128, 2), (128, 8), (128, 1), (64, 8), (64, 1)])
def test_paged_prefill(gpu, D, G, version):
    hkv = 2
    hq = hkv * G
    # (context already cached, new query tokens): plain prefill, chunked continuation, 1-token tail
    specs = [(0, 77), (300, 45), (16, 1), (0, 130), (33, 200)]
    seq_lens = [c + n for c, n in specs]
    kv, bt = _paged_setup(seq_lens, hkv, D, device=gpu)
    qsl = [0]
    for _, n in specs:
        qsl.append(qsl[-1] + n)
    T = qsl[-1]
    q = torch.randn(T, hq, D, device=gpu, dtype=torch.bfloat16)
    qsl_t = torch.tensor(qsl, dtype=torch.int32)
    sl = torch.tensor(seq_lens, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    out = ops.paged_attention_prefill(q, kv[:, 1], bt.to(gpu), qsl_t.to(gpu), sl.to(gpu), scale,
                                      max(n for _, n in specs), version=version)
    exp = ref.paged_attention(q.cpu(), kv[:, 1].cpu(), bt, qsl_t, sl, scale)
    _close(out, exp, 0.03, 0.03, f"prefill v{version}")


@pytest.mark.parametrize("version", [2, 3])
def test_prefill_softmax_rescale_spike(gpu, version):
    """Force the online-softmax rescale: one key much larger late in the sequence (rule 26)."""
    D, G, hkv = 64, 4, 1
    lens = [256]
    kv, bt = _paged_setup(lens, hkv, D, device=gpu)
    q = torch.randn(256, G, D, device=gpu, dtype=torch.bfloat16)
    nb_idx = int(bt[0, 200 // 16])
    kv[nb_idx, 1, 0, 0, 200 % 16, :] = q[255, 0] * 4  # spike key 200 for query 255
    out = ops.paged_attention_prefill(q, kv[:, 1], bt.to(gpu), torch.tensor([0, 256], dtype=torch.int32, device=gpu),
                                      torch.tensor(lens, dtype=torch.int32, device=gpu), 0.125, 256, version=version)
    exp = ref.paged_attention(q.cpu(), kv[:, 1].cpu(), bt, torch.tensor([0, 256], dtype=torch.int32),
                              torch.tensor(lens, dtype=torch.int32), 0.125)
    _close(out, exp, 0.03, 0.03, "prefill-spike")


# v3 softmax variants (attention_prefill.hip VAR bits: 1 biased reference + overflow redo, 2 row sum
# on the matrix pipe, 4 persistent -m accumulator block), launched as version 0x100 | VAR at G = 4
@pytest.mark.parametrize("var", [0, 1, 2, 4, 6, 7, 8, 10, 12, 14, 16, 32, 36, 64, 66, 128, 256, 1024, 1280])
@pytest.mark.parametrize("D", [64, 128])
def test_paged_prefill_softmax_variants(gpu, D, var):
    G, hkv = 4, 2
    specs = [(0, 77), (300, 45), (16, 1), (0, 130), (33, 200)]
    seq_lens = [c + n for c, n in specs]
    kv, bt = _paged_setup(seq_lens, hkv, D, device=gpu)
    qsl = [0]
    for _, n in specs:
        qsl.append(qsl[-1] + n)
    q = torch.randn(qsl[-1], hkv * G, D, device=gpu, dtype=torch.bfloat16)
    qsl_t, sl = torch.tensor(qsl, dtype=torch.int32), torch.tensor(seq_lens, dtype=torch.int32)
    out = ops.paged_attention_prefill(q, kv[:, 1], bt.to(gpu), qsl_t.to(gpu), sl.to(gpu), 1 / math.sqrt(D),
                                      max(n for _, n in specs), version=0x100 + var)
    exp = ref.paged_attention(q.cpu(), kv[:, 1].cpu(), bt, qsl_t, sl, 1 / math.sqrt(D))
    _close(out, exp, 0.03, 0.03, f"prefill var {var}")


@pytest.mark.parametrize("var,fp8", [(128, False), (128, True), (256, False)])
@pytest.mark.parametrize("D,G", [(64, 4), (128, 4), (64, 1), (128, 8)])
def test_paged_prefill_split(gpu, D, G, var, fp8):
    """VAR 128: q-tiles with >= 8 key tiles run as two workgroups over the two halves of their key
    range, merged by the second to finish.  VAR 256: each workgroup runs a heavy and a light q-tile of
    its sequence.  Long prompts, a prefix-cache hit, a short chunk over a long
    context and a short prompt (unsplit) in one launch; launched three times, the output must not change
    (the tile counters are never reset: the ticket parity names the merging half)."""
    hkv = 2
    specs = [(0, 2000), (1500, 700), (3000, 5), (0, 100)]
    seq_lens = [c + n for c, n in specs]
    kv, bt = _paged_setup(seq_lens, hkv, D, device=gpu)
    ks, vs = (0.5, 0.25) if fp8 else (1.0, 1.0)
    cache = _fp8_cache(kv, 1.0) if fp8 else kv
    qsl = [0]
    for _, n in specs:
        qsl.append(qsl[-1] + n)
    q = torch.randn(qsl[-1], hkv * G, D, device=gpu, dtype=torch.bfloat16)
    qsl_t, sl = torch.tensor(qsl, dtype=torch.int32), torch.tensor(seq_lens, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    outs = [ops.paged_attention_prefill(q, cache[:, 1], bt.to(gpu), qsl_t.to(gpu), sl.to(gpu), scale,
                                        max(n for _, n in specs), version=0x100 + var, k_scale=ks, v_scale=vs)
            for _ in range(3)]
    exp = ref.paged_attention(q.cpu(), cache[:, 1].cpu(), bt, qsl_t, sl, scale, ks, vs)
    _close(outs[0], exp, 0.03, 0.03, f"prefill var {var} D{D} G{G} fp8={fp8}")
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    base = ops.paged_attention_prefill(q, cache[:, 1], bt.to(gpu), qsl_t.to(gpu), sl.to(gpu), scale,
                                       max(n for _, n in specs), version=0x100, k_scale=ks, v_scale=vs)
    # the unsplit kernel on the same inputs: the split changes only rounding
    assert (outs[0].float() - base.float()).abs().max().item() < 0.03


@pytest.mark.parametrize("factor", [4, 12])
@pytest.mark.parametrize("var", [0, 1, 7, 8, 14, 32])
def test_prefill_softmax_variant_spikes(gpu, var, factor):
    """Late keys far above every earlier score of their rows: at factor 12 the score passes the running
    max by ~140 (log2 units), past exp2's f32 range, so VAR & 1 must take its redo path; several rows
    and both 32-key halves of a tile spike, one row twice (rule 26: the branch is data-dependent)."""
    torch.manual_seed(0)  # the bf16 rounding of near-one-hot rows sits close to the tolerance on some draws
    D, G, hkv = 64, 4, 1
    lens = [256]
    kv, bt = _paged_setup(lens, hkv, D, device=gpu)
    q = torch.randn(256, G, D, device=gpu, dtype=torch.bfloat16)
    for key, (tok, head) in ((200, (255, 0)), (130, (140, 2)), (161, (200, 1)), (230, (255, 0))):
        nb_idx = int(bt[0, key // 16])
        kv[nb_idx, 1, 0, 0, key % 16, :] = q[tok, head] * factor
    qsl = torch.tensor([0, 256], dtype=torch.int32)
    sl = torch.tensor(lens, dtype=torch.int32)
    out = ops.paged_attention_prefill(q, kv[:, 1], bt.to(gpu), qsl.to(gpu), sl.to(gpu), 0.125, 256,
                                      version=0x100 | var)
    assert torch.isfinite(out).all()
    exp = ref.paged_attention(q.cpu(), kv[:, 1].cpu(), bt, qsl, sl, 0.125)
    _close(out, exp, 0.03, 0.03, f"prefill-spike var {var} x{factor}")


# ---- fp8 (e4m3fn) KV cache: the cache bytes are shared by kernel and reference, so attention must
# match the reference over the same dequantised values; the write path is checked byte-for-byte
# against torch's e4m3fn rounding (off by one ulp allowed where f32 rounding of RoPE differs).
def _fp8_cache(kv_bf16, scale=1.0):
    return (kv_bf16.float() / scale).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)


@pytest.mark.parametrize("D,hq,hkv,qknorm", [(64, 32, 8, False), (128, 16, 8, True)])
@pytest.mark.parametrize("kscale", [1.0, 0.05])
def test_rope_and_cache_fp8(gpu, D, hq, hkv, qknorm, kscale):
    T, L, nb = 37, 2, 20
    cos_sin = ref.build_cos_sin_cache(D, 4096, 500000.0, None, device=gpu)
    qkv = (torch.randn(T, (hq + 2 * hkv) * D, device=gpu) * 3).to(torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=gpu)
    slots = torch.randperm(nb * 16, device=gpu)[:T]
    slots[5] = -1
    qn = (1 + 0.1 * torch.randn(D, device=gpu)).bfloat16() if qknorm else None
    kn = (1 + 0.1 * torch.randn(D, device=gpu)).bfloat16() if qknorm else None
    kv = torch.zeros(nb, L, 2, hkv, 16, D, device=gpu, dtype=torch.uint8)
    kv_ref = kv.clone().cpu()
    q = ops.rope_and_cache(qkv, hq, hkv, D, pos, cos_sin, kv[:, 1], slots, qn, kn, 1e-6, k_scale=kscale,
                           v_scale=kscale)
    qs, ks = hq * D, hkv * D
    c = qkv.cpu()
    q_ref = ref.rope_and_cache(c[:, :qs].reshape(T, hq, D), c[:, qs:qs + ks].reshape(T, hkv, D),
                               c[:, qs + ks:].reshape(T, hkv, D), pos.cpu(), cos_sin.cpu(), kv_ref[:, 1],
                               slots.cpu(), None if qn is None else qn.cpu(), None if kn is None else kn.cpu(), 1e-6,
                               k_scale=kscale, v_scale=kscale)
    _close(q, q_ref, 0.03, 0.02, "q")
    got = kv.cpu().view(torch.float8_e4m3fn).float()
    exp = kv_ref.view(torch.float8_e4m3fn).float()
    # e4m3 has 3 mantissa bits: one ulp is 12.5 % relative.  V (bf16 in, no RoPE) at scale 1 is
    # exact; otherwise x * (1/scale) vs x / scale may straddle a rounding tie: one ulp at most
    if kscale == 1.0:
        _close(got[:, 1, 1], exp[:, 1, 1], 0.0, 0.0, "v bytes")
    for kvi, name in ((0, "k"), (1, "v")):
        _close(got[:, 1, kvi], exp[:, 1, kvi], 2 ** -9, 0.13, f"{name} bytes")
        ulp = (kv.cpu()[:, 1, kvi].view(torch.int8).int() - kv_ref[:, 1, kvi].view(torch.int8).int()).abs()
        assert ulp.max().item() <= 1, f"{name}: {ulp.max().item()} ulp"
    assert kv[:, 0].sum().item() == 0  # other layer untouched


@pytest.mark.parametrize("impl", [1, 2])
@pytest.mark.parametrize("D,G", [(64, 4), (128, 2), (128, 8), (64, 1)])
@pytest.mark.parametrize("scales", [(1.0, 1.0), (0.02, 0.05)])
def test_paged_decode_fp8(gpu, D, G, scales, impl):
    ks, vs = scales
    hkv, lens = 2, [1, 17, 513, 2000, 4096]
    kv, bt = _paged_setup(lens, hkv, D, device=gpu)
    kv8 = _fp8_cache(kv * (ks * 4), ks)  # stored values ~ N(0, 2): the fp8 grid is coarse there
    B = len(lens)
    q = torch.randn(B, hkv * G, D, device=gpu, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    out = ops.paged_attention_decode(q, kv8[:, 1], bt.to(gpu), sl.to(gpu), scale, max(lens), k_scale=ks, v_scale=vs,
                                     impl=impl)
    exp = ref.paged_attention_decode(q.cpu(), kv8[:, 1].cpu(), bt, sl, scale, ks, vs)
    _close(out, exp, 0.02 * max(1.0, exp.abs().max().item()), 0.02, "decode fp8")


@pytest.mark.parametrize("D,G", [(64, 4), (128, 2), (128, 8)])
def test_paged_prefill_fp8(gpu, D, G):
    hkv, ks, vs = 2, 0.5, 0.25
    specs = [(0, 77), (300, 45), (16, 1), (33, 200)]
    seq_lens = [c + n for c, n in specs]
    kv, bt = _paged_setup(seq_lens, hkv, D, device=gpu)
    kv8 = _fp8_cache(kv, 1.0)
    qsl = [0]
    for _, n in specs:
        qsl.append(qsl[-1] + n)
    q = torch.randn(qsl[-1], hkv * G, D, device=gpu, dtype=torch.bfloat16)
    qsl_t = torch.tensor(qsl, dtype=torch.int32)
    sl = torch.tensor(seq_lens, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    # version 2 requested: the fp8 cache always runs v3
    out = ops.paged_attention_prefill(q, kv8[:, 1], bt.to(gpu), qsl_t.to(gpu), sl.to(gpu), scale,
                                      max(n for _, n in specs), version=2, k_scale=ks, v_scale=vs)
    exp = ref.paged_attention(q.cpu(), kv8[:, 1].cpu(), bt, qsl_t, sl, scale, ks, vs)
    _close(out, exp, 0.03, 0.03, "prefill fp8")


@pytest.mark.parametrize("dtype,V", [(torch.float32, 128256), (torch.bfloat16, 128256), (torch.bfloat16, 1001)])
def test_sample_greedy(gpu, dtype, V):
    B = 16
    logits = torch.randn(B, V, device=gpu).to(dtype)
    logits[3, 77] = 50.0
    z = torch.zeros(B, device=gpu)
    ids = ops.sample(logits, z, torch.ones(B, device=gpu), torch.zeros(B, dtype=torch.int32, device=gpu),
                     torch.arange(B, device=gpu), torch.zeros(B, dtype=torch.int64, device=gpu))
    assert torch.equal(ids.cpu(), logits.argmax(-1).cpu())
    assert int(ids[3]) == 77


@pytest.mark.parametrize("dtype,V", [(torch.float32, 32000), (torch.bfloat16, 32000), (torch.bfloat16, 128256)])
@pytest.mark.parametrize("top_p,top_k", [(1.0, 0), (0.9, 0), (1.0, 50), (0.8, 20)])
def test_sample_matches_reference(gpu, top_p, top_k, dtype, V):
    """bf16 rows take the register-resident kernel (row loaded once, bisection passes on registers;
    V = 32000 pads the last 16-byte slots), fp32 rows the memory form."""
    B = 24
    logits = (torch.randn(B, V, device=gpu) * 3).to(dtype)
    t = torch.full((B,), 0.7, device=gpu)
    tp = torch.full((B,), top_p, device=gpu)
    tk = torch.full((B,), top_k, dtype=torch.int32, device=gpu)
    seeds = torch.arange(100, 100 + B, device=gpu)
    steps = torch.full((B,), 3, dtype=torch.int64, device=gpu)
    ids = ops.sample(logits, t, tp, tk, seeds, steps).cpu()
    exp = ref.sample(logits.cpu(), t.cpu(), tp.cpu(), tk.cpu(), seeds.cpu(), steps.cpu())
    agree = (ids == exp).float().mean().item()
    assert agree >= 0.9, f"only {agree:.2f} of rows agree with the reference sampler"


def test_sample_distribution(gpu):
    """Gumbel-max frequencies follow softmax(z/T)."""
    V, N = 8, 4000
    z = torch.tensor([2.0, 1.0, 0.5, 0.0, -1.0, -2.0, -3.0, -4.0], device=gpu)
    logits = z.unsqueeze(0).repeat(N, 1).contiguous()
    t = torch.ones(N, device=gpu)
    ids = ops.sample(logits, t, torch.ones(N, device=gpu), torch.zeros(N, dtype=torch.int32, device=gpu),
                     torch.arange(N, device=gpu), torch.zeros(N, dtype=torch.int64, device=gpu)).cpu()
    freq = torch.bincount(ids, minlength=V).float() / N
    p = torch.softmax(z.cpu(), -1)
    assert (freq - p).abs().max().item() < 0.03


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("k", [0, 1, 5, 20])
def test_logprobs_matches_reference(gpu, dtype, k):
    """Log-prob kernel vs fp32 log_softmax + stable top-k, on a padded-vocab row view (TP lm_head)."""
    B, V, Vpad = 12, 128256, 128256 + 64
    full = (torch.randn(B, Vpad, device=gpu) * 4).to(dtype)
    logits = full[:, :V]
    rows = torch.tensor([0, 3, 4, 11], device=gpu)
    toks = torch.tensor([5, 77, 128255, 1000], device=gpu)
    tlp, tid, tv = ops.logprobs(logits, rows, toks, k)
    etlp, etid, etv = ref.logprobs(logits.cpu(), rows.cpu(), toks.cpu(), k)
    _close(tlp, etlp, 1e-3, 1e-3, "token logprob")
    assert tid.shape == (4, k) and tv.shape == (4, k)
    if k:
        _close(tv, etv, 1e-3, 1e-3, "top logprobs")
        # bf16 logits tie often: compare ids where the reference values are distinct
        distinct = torch.cat([etv[:, :-1] != etv[:, 1:], torch.ones(4, 1, dtype=torch.bool)], 1)
        distinct &= torch.cat([torch.ones(4, 1, dtype=torch.bool), etv[:, 1:] != etv[:, :-1]], 1)
        assert torch.equal(tid.cpu()[distinct], etid[distinct])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_penalties_match_reference(gpu, dtype):
    """Penalty kernel vs the reference on random histories (repeats, prompt/output split, rows
    with neutral penalties untouched), on a padded-vocab view."""
    B, V, L, rows_total = 6, 128256, 300, 10
    g = torch.Generator().manual_seed(3)
    full = (torch.randn(B, V + 64, generator=g) * 3).to(dtype)
    hist = torch.randint(0, 2000, (rows_total, L), generator=g, dtype=torch.int32)  # small range: many repeats
    srows = torch.tensor([3, 0, 9, 5, 1, 7])
    hlen = torch.tensor([300, 1, 150, 64, 0, 299], dtype=torch.int32)
    plen = torch.tensor([100, 1, 150, 0, 0, 10], dtype=torch.int32)
    rep = torch.tensor([1.3, 1.0, 1.0, 0.8, 1.5, 1.0])
    freq = torch.tensor([0.5, 0.0, 0.2, -0.3, 0.0, 0.0])
    pres = torch.tensor([0.25, 0.0, 1.0, 0.0, 0.5, 0.0])
    exp = full[:, :V].clone()
    ref.apply_penalties(exp, hist, srows, hlen, plen, rep, freq, pres)
    got_full = full.to(gpu)
    got = got_full[:, :V]
    ops.apply_penalties(got, hist.to(gpu), srows.to(gpu), hlen.to(gpu), plen.to(gpu), rep.to(gpu), freq.to(gpu),
                        pres.to(gpu))
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    _close(got, exp, tol, tol, "penalized logits")
    assert torch.equal(got_full[:, V:].cpu(), full[:, V:])  # padding columns untouched
    assert torch.equal(got[5].cpu(), full[5, :V]) and torch.equal(got[1].cpu(), full[1, :V])  # neutral rows


def test_moe_topk_softmax(gpu):
    T, E, K = 100, 8, 2
    g = torch.Generator().manual_seed(0)
    # distinct values per row (random bf16 logits tie often, and tie order is not part of the contract)
    logits = (torch.stack([torch.randperm(E, generator=g) for _ in range(T)]).float() * 0.37 - 1.2)
    logits = logits.to(device=gpu, dtype=torch.bfloat16)
    w, ids = ops.moe_topk_softmax(logits, K)
    ew, eids = ref.moe_topk_softmax(logits.cpu(), K)
    assert torch.equal(ids.cpu(), eids)
    _close(w, ew, 1e-3, 1e-3, "topk weights")


def test_moe_align(gpu):
    T, K, E = 300, 2, 8
    ids = torch.randint(0, E, (T, K), dtype=torch.int32, device=gpu)
    offs = torch.empty(E // 2 + 1, dtype=torch.int32, device=gpu)
    perm = torch.full((T * K,), -1, dtype=torch.int32, device=gpu)
    inv = torch.empty(T * K, dtype=torch.int32, device=gpu)
    ops.ext().moe_align(offs, perm, ids, 4, E // 2, inv)  # local experts 4..7
    flat = ids.flatten().cpu()
    o = offs.cpu().tolist()
    p = perm.cpu()
    for e in range(E // 2):
        rows = p[o[e]:o[e + 1]]
        exp = (flat == e + 4).nonzero().flatten()
        assert torch.equal(rows.long(), exp), f"expert {e}"
    iv = inv.cpu().long()
    local = flat >= 4
    assert torch.equal(p[iv[local]].long(), torch.arange(T * K)[local])  # inverse permutation
    assert (iv[~local] == -1).all()


@pytest.mark.parametrize("split", [2, 3, 6])  # K = 384: 6 K-steps of 64
def test_moe_grouped_gemm_split_k(gpu, split):
    """Split-K down projection: the fp32 slices summed by moe_combine_partials equal the unsplit
    GEMM followed by moe_combine."""
    T, K, E, H, I = 37, 2, 4, 256, 384
    ids = torch.randint(0, E, (T, K), device=gpu, dtype=torch.int32)
    offs = torch.empty(E + 1, dtype=torch.int32, device=gpu)
    perm = torch.full((T * K,), -1, dtype=torch.int32, device=gpu)
    inv = torch.empty(T * K, dtype=torch.int32, device=gpu)
    ops.ext().moe_align(offs, perm, ids, 0, E, inv)
    h = torch.randn(T * K, I, device=gpu, dtype=torch.bfloat16)
    w2 = torch.randn(E, H, I, device=gpu, dtype=torch.bfloat16) * 0.05
    w = torch.rand(T, K, device=gpu)
    ys = torch.empty(T * K, H, device=gpu, dtype=torch.bfloat16)
    assert ops.ext().moe_grouped_gemm(ys, h, w2, offs, False)
    ref_out = torch.empty(T, H, device=gpu, dtype=torch.bfloat16)
    ops.ext().moe_combine(ref_out, ys, w, inv)
    part = torch.empty(split, T * K, H, device=gpu, dtype=torch.float32)
    assert ops.ext().moe_grouped_gemm(ys, h, w2, offs, False, split, part)
    out = torch.empty(T, H, device=gpu, dtype=torch.bfloat16)
    ops.ext().moe_combine_partials(out, part, w, inv)
    _close(out, ref_out, 0.02, 0.02, f"split-K {split}")


@pytest.mark.parametrize("split", [2, 4])
def test_moe_gate_up_split_k(gpu, split):
    """Split-K gate_up: fp32 slices over [gate; up] + silu_mul_partials equal the fused SiLU GEMM."""
    T, K, E, H, I = 29, 2, 3, 256, 384
    ids = torch.randint(0, E, (T, K), device=gpu, dtype=torch.int32)
    offs = torch.empty(E + 1, dtype=torch.int32, device=gpu)
    perm = torch.full((T * K,), -1, dtype=torch.int32, device=gpu)
    ops.ext().moe_align(offs, perm, ids, 0, E)
    xs = torch.randn(T * K, H, device=gpu, dtype=torch.bfloat16)
    w13 = torch.randn(E, 2 * I, H, device=gpu, dtype=torch.bfloat16) * 0.05
    h_ref = torch.empty(T * K, I, device=gpu, dtype=torch.bfloat16)
    assert ops.ext().moe_grouped_gemm(h_ref, xs, w13, offs, True)
    part = torch.empty(split, T * K, 2 * I, device=gpu, dtype=torch.float32)
    assert ops.ext().moe_grouped_gemm(h_ref.new_empty(0, 2 * I), xs, w13, offs, False, split, part)
    h = torch.empty_like(h_ref)
    ops.ext().silu_mul_partials(h, part)
    rows = int(offs[-1])
    _close(h[:rows], h_ref[:rows], 0.02, 0.02, f"gate_up split {split}")


def test_moe_combine(gpu):
    """K17: each token sums its top-k expert rows (gathered through the inverse permutation) with
    the routing weights; rows owned by other ranks (inv < 0) contribute nothing."""
    T, K, H, R = 77, 2, 512, 120
    ys = torch.randn(R, H, device=gpu, dtype=torch.bfloat16)
    w = torch.rand(T, K, device=gpu)
    inv = torch.randint(-1, R, (T * K,), device=gpu, dtype=torch.int32)
    out = torch.empty(T, H, device=gpu, dtype=torch.bfloat16)
    ops.ext().moe_combine(out, ys, w, inv)
    yv = torch.cat([ys.float().cpu(), torch.zeros(1, H)])
    idx = inv.cpu().long().view(T, K)
    exp = (yv[torch.where(idx < 0, R, idx)] * w.cpu().unsqueeze(-1)).sum(1)
    _close(out, exp, 0.02, 0.01, "moe_combine")


@pytest.mark.parametrize("T", [64, 300, 700])
def test_moe_experts_gpu_vs_ref(gpu, T):
    """T = 700 takes the prefill path (per-expert hipBLASLt over gathered rows, K17 combine)."""
    H, I, E, K = 256, 192, 4, 2
    x = torch.randn(T, H, device=gpu, dtype=torch.bfloat16)
    w13 = torch.randn(E, 2 * I, H, device=gpu, dtype=torch.bfloat16) * 0.05
    w2 = torch.randn(E, H, I, device=gpu, dtype=torch.bfloat16) * 0.05
    logits = torch.randn(T, E, device=gpu, dtype=torch.bfloat16)
    tw, tid = ops.moe_topk_softmax(logits, K)
    out = ops.moe_experts(x, w13, w2, tw, tid, 0)
    exp = ref.moe_experts(x.cpu(), w13.cpu(), w2.cpu(), tw.cpu(), tid.cpu(), 0)
    _close(out, exp, 0.02, 0.03, "moe")


@pytest.mark.parametrize("layout", ["fixed", "variable", "ipc"])
def test_moe_a2a_dispatch_gpu(gpu, layout):
    """All-to-all expert dispatch (mxserve/parallel/expert.py) on one rank: slice/route/dispatch/
    grouped-GEMM/combine through the HIP kernels vs the fp32 reference MoE."""
    from mxserve.parallel.expert import moe_a2a
    T, H, I, E, K = 96, 256, 192, 8, 2
    x = torch.randn(T, H, device=gpu, dtype=torch.bfloat16)
    gate = torch.randn(E, H, device=gpu, dtype=torch.bfloat16) * 0.1
    w13 = torch.randn(E, 2 * I, H, device=gpu, dtype=torch.bfloat16) * 0.05
    w2 = torch.randn(E, H, I, device=gpu, dtype=torch.bfloat16) * 0.05
    out = moe_a2a(x, gate, w13, w2, K, 0, 1, None, force_layout=layout)
    tw, tid = ops.moe_topk_softmax(torch.nn.functional.linear(x, gate), K)
    exp = ref.moe_experts(x.cpu(), w13.cpu(), w2.cpu(), tw.cpu(), tid.cpu(), 0)
    _close(out, exp, 0.02, 0.03, "moe a2a")


def test_copy_blocks(gpu):
    src = torch.randn(10, 4, 512, device=gpu, dtype=torch.bfloat16)
    dst = torch.zeros(12, 4, 512, device=gpu, dtype=torch.bfloat16)
    s_ids = torch.tensor([1, 5, 9], dtype=torch.int32, device=gpu)
    d_ids = torch.tensor([0, 11, 3], dtype=torch.int32, device=gpu)
    ops.ext().copy_blocks(dst.data_ptr(), src, s_ids, d_ids, src[0].numel() * 2)
    torch.cuda.synchronize()
    for s, d in zip(s_ids.tolist(), d_ids.tolist()):
        assert torch.equal(dst[d], src[s])
    assert dst[1].abs().sum().item() == 0


@pytest.mark.parametrize("N,K,epi", [(3072, 2048, 0), (2048, 8192, 0), (16384, 2048, 1), (2048, 2048, 0),
                                     (28672, 4096, 1), (128256, 2048, 0)])
@pytest.mark.parametrize("M", [1, 3, 16, 24, 33, 64, 100, 192, 256])
def test_decode_gemm_all_configs(gpu, M, N, K, epi):
    """Every tiling / split-K configuration of the decode projection kernel vs an fp32 reference,
    plain (qkv / o / down / lm_head) and with SiLU*mul fused (gate_up: w = [gate; up])."""
    from mxserve.ops import decode_gemm
    x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=gpu) * K ** -0.5).to(torch.bfloat16)
    y = x.float() @ w.float().t()
    want = torch.nn.functional.silu(y[:, :N // 2]) * y[:, N // 2:] if epi else y
    cands = decode_gemm.candidates(M, N, K, epi)
    assert cands
    part = torch.empty(max(decode_gemm.SPLITS) * M * N, dtype=torch.float32, device=gpu)
    reg = [c for c in cands if isinstance(c[0], int)]
    assert any(c[4] for c in reg) or M <= 16, "LDS-form configurations are among the candidates"
    big = N * K * 2 >= decode_gemm.MT_SMALL_M_MIN_BYTES
    assert any(c[0] == "mt" for c in cands) == (M >= decode_gemm.MT_MIN_M or big)
    assert any(c[0] == "sk" for c in cands) == (M <= 64 and N % (32 if epi else 16) == 0 and
                                                 K % (512 if M <= 16 else 256) == 0)
    decode_gemm.TABLE.part = part
    for c in cands:
        out = torch.full((M, N // 2 if epi else N), float("nan"), device=gpu, dtype=torch.bfloat16)
        if c[0] == "mt":
            assert ops.ext().mt_gemm(out, x, w, part, *c[1:6], epi, None, c[6] if len(c) > 6 else 0)
        elif c[0] in ("sk", "pf", "gv"):
            assert decode_gemm.TABLE.run(out, x, w, c, epi)
        else:
            assert ops.ext().decode_gemm(out, x, w, part, *c[:4], epi, c[4])
        _close(out, want, atol=2e-2, rtol=2e-2, name=f"decode gemm {M}x{N}x{K} epi{epi} cfg {c}")


@pytest.mark.parametrize("N,K,epi", [(3072, 2048, 0), (2048, 8192, 0), (16384, 2048, 1), (1024, 512, 1)])
@pytest.mark.parametrize("M", [1, 33, 64, 100, 192, 256, 300, 640])
def test_mt_gemm_all_layouts(gpu, M, N, K, epi):
    """Every wave layout and split-K of the medium-M kernel (gemm_decode.hip mt_gemm_kernel, glds
    staging) vs an fp32 reference, including partial row tiles, several row tiles (prefill-sized M)
    and a K of 2 k-groups per slice; an asymmetric W catches a transposed store."""
    from mxserve.ops import decode_gemm
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N)
    x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16, generator=g)
    w = (torch.randn(N, K, device=gpu, generator=g) * K ** -0.5).to(torch.bfloat16)
    w[:, : K // 2] *= torch.linspace(0.5, 2.0, N, device=gpu).to(torch.bfloat16)[:, None]
    y = x.float() @ w.float().t()
    want = torch.nn.functional.silu(y[:, :N // 2]) * y[:, N // 2:] if epi else y
    part = torch.empty(8 * M * N, dtype=torch.float32, device=gpu)
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=gpu)
    ran = 0
    for lay in decode_gemm.MT_LAYOUTS:
        for sk in (1, 2, 4):
            for fused, order in (((False, 0), (True, 0), (False, 1), (True, 1)) if sk > 1 else ((False, 0), (False, 1))):
                out = torch.full((M, N // 2 if epi else N), float("nan"), device=gpu, dtype=torch.bfloat16)
                for _ in range(2 if fused else 1):  # the second launch reuses the counters the first re-armed
                    if not ops.ext().mt_gemm(out, x, w, part, *lay, sk, epi, cnt if fused else None, order):
                        break
                else:
                    ran += 1
                    _close(out, want, atol=2e-2, rtol=2e-2,
                           name=f"mt gemm {M}x{N}x{K} epi{epi} {lay} sk{sk} fused-reduce {fused} order {order}")
    assert ran >= 8
    assert int(cnt.abs().sum().item()) == 0, "every launch leaves the tile counters zero"


def test_decode_gemm_tuner_and_dispatch(gpu, monkeypatch):
    """The graph-time tuner times the kernel against hipBLASLt per (bucket, projection), keeps a winner
    only when it matches hipBLASLt, and ops.linear / ops.gate_up_silu then follow the table."""
    from mxserve.ops import decode_gemm
    monkeypatch.setattr(decode_gemm, "MODE", "auto")
    monkeypatch.setattr(decode_gemm, "MAX_TUNE_M", 256)
    monkeypatch.setenv("MXS_RETUNE", "1")  # measure, whatever the packaged table holds
    monkeypatch.delenv("MXS_TUNED_SAVE", raising=False)
    w1 = (torch.randn(2048, 2048, device=gpu) * 0.02).to(torch.bfloat16)
    w2 = (torch.randn(2 * 8192, 2048, device=gpu) * 0.02).to(torch.bfloat16)
    w3 = (torch.randn(3072, 2048, device=gpu) * 0.02).to(torch.bfloat16)
    rows = decode_gemm.tune({"o": (w1, 0, ("add_norm",)), "gate_up": (w2, 1), "qkv": (w3, 0, ("rope", 32, 8, 64))},
                            [1, 8, 64, 256], gpu)
    assert len(rows) == 12 and all(r["us"] <= r["hipblaslt_us"] for r in rows)
    assert {r["epilogue"] for r in rows} == {"+norm", "+rope", None}
    for M in (1, 64):
        x = torch.randn(M, 2048, device=gpu, dtype=torch.bfloat16)
        _close(ops.linear(x, w1), x.float() @ w1.float().t(), 2e-2, 2e-2, "tuned linear")
        y = x.float() @ w2.float().t()
        _close(ops.gate_up_silu(x, w2), torch.nn.functional.silu(y[:, :8192]) * y[:, 8192:], 2e-2, 2e-2,
               "tuned gate_up")
        res = torch.randn(M, 2048, device=gpu, dtype=torch.bfloat16)
        nw = torch.ones(2048, device=gpu, dtype=torch.bfloat16)
        r2 = res.clone()
        h, _ = ops.linear_add_rms_norm(x, w1, r2, nw, 1e-5)
        r_want = (x.float() @ w1.float().t()).to(torch.bfloat16).float() + res.float()
        _close(r2, r_want, 3e-2, 2e-2, "tuned o + residual")
        _close(h, r_want * torch.rsqrt(r_want.pow(2).mean(-1, keepdim=True) + 1e-5), 3e-2, 3e-2, "tuned o + norm")


def test_decode_gemm_rejects_untiled_shapes(gpu):
    x = torch.randn(8, 1000, device=gpu, dtype=torch.bfloat16)  # K not a multiple of 32
    w = torch.randn(1056, 1000, device=gpu, dtype=torch.bfloat16)
    out = torch.empty(8, 1056, device=gpu, dtype=torch.bfloat16)
    assert not ops.ext().decode_gemm(out, x, w, None, 1, 2, 1, 1, 0)
    w2 = torch.randn(1000, 1024, device=gpu, dtype=torch.bfloat16)  # N not a multiple of the tile
    x2 = torch.randn(8, 1024, device=gpu, dtype=torch.bfloat16)
    assert not ops.ext().decode_gemm(torch.empty(8, 1000, device=gpu, dtype=torch.bfloat16), x2, w2, None, 1, 4, 1,
                                     1, 0)


@pytest.mark.parametrize("counts", [[0, 5, 300, 1], [128, 129, 0, 3], [1, 1, 1, 1]])
@pytest.mark.parametrize("silu", [False, True])
def test_moe_grouped_gemm(gpu, counts, silu):
    E, N, K = len(counts), 256, 320
    rows = sum(counts) + 37  # extra rows past the routed count must be left alone
    g = torch.Generator(device="cuda").manual_seed(sum(counts) + silu)
    x = torch.randn(rows, K, device=gpu, dtype=torch.bfloat16, generator=g)
    w = (torch.randn(E, N, K, device=gpu, dtype=torch.bfloat16, generator=g) * 0.05).to(torch.bfloat16)
    offs = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int32, device=gpu)
    y = torch.full((rows, N // 2 if silu else N), 7.0, device=gpu, dtype=torch.bfloat16)
    assert ops.ext().moe_grouped_gemm(y, x, w, offs, silu)
    o = offs.tolist()
    for e in range(E):
        a, b = o[e], o[e + 1]
        if b == a:
            continue
        ref_y = x[a:b].float() @ w[e].float().t()
        if silu:
            gt, up = ref_y[:, :N // 2], ref_y[:, N // 2:]
            ref_y = gt * torch.sigmoid(gt) * up
        _close(y[a:b], ref_y, atol=3e-2, rtol=3e-2, name=f"expert {e}")
    assert torch.all(y[o[-1]:] == 7.0), "rows past the routed count were written"


@pytest.mark.parametrize("counts", [[0, 5, 70, 1], [16, 17, 0, 33], [1, 1, 1, 1], [130, 0, 0, 2]])
@pytest.mark.parametrize("silu", [False, True])
def test_moe_decode_gemm_all_configs(gpu, counts, silu):
    """Grouped form of the decode GEMM kernel (K16 at decode batches) in every configuration the
    launcher takes: each expert's rows vs fp32, rows past the routed count untouched, split-K slabs."""
    from mxserve.ops import decode_gemm as dg
    E, N, K = len(counts), 512, 1024
    R = sum(counts) + 9
    rows_max = max(counts)
    g = torch.Generator(device="cuda").manual_seed(sum(counts) + silu)
    x = torch.randn(R, K, device=gpu, dtype=torch.bfloat16, generator=g)
    w = (torch.randn(E, N, K, device=gpu, dtype=torch.bfloat16, generator=g) * 0.05).to(torch.bfloat16)
    offs = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int32, device=gpu)
    o = offs.tolist()
    refs = {}
    for e in range(E):
        a, b = o[e], o[e + 1]
        if b > a:
            refs[e] = x[a:b].float() @ w[e].float().t()
    epi = int(silu)
    ran = 0
    for cfg in dg.candidates(rows_max, N, K, epi, all_mf=True, mt=False):
        mf, nf, wm, sk, lu = cfg
        if wm > 2:
            continue
        y = torch.full((R, N // 2 if silu else N), 7.0, device=gpu, dtype=torch.bfloat16)
        part = torch.zeros(sk, R, N, device=gpu, dtype=torch.float32) if sk > 1 else None
        assert ops.ext().moe_decode_gemm(y, x, w, offs, part, rows_max, mf, nf, wm, sk, epi, lu), cfg
        ran += 1
        for e, r in refs.items():
            a, b = o[e], o[e + 1]
            if sk > 1:
                got = part[:, a:b].sum(0)
                _close(got, r, atol=3e-2, rtol=3e-2, name=f"expert {e} cfg {cfg} slabs")
                continue
            exp = r
            if silu:
                gt, up = r[:, :N // 2], r[:, N // 2:]
                exp = gt * torch.sigmoid(gt) * up
            _close(y[a:b], exp, atol=3e-2, rtol=3e-2, name=f"expert {e} cfg {cfg}")
        if sk == 1:
            assert torch.all(y[o[-1]:] == 7.0), f"rows past the routed count were written ({cfg})"
    assert ran >= 6 and any(c[4] for c in dg.candidates(rows_max, N, K, epi, all_mf=True, mt=False))


@pytest.mark.parametrize("T,offset", [(1, 0), (7, 0), (64, 0), (200, 0), (40, 2)])
def test_moe_experts_decode_kernel_path(gpu, monkeypatch, T, offset):
    """fused_experts at decode batches runs both expert GEMMs on the grouped decode kernel (split-K
    slabs summed by silu_mul_partials / moe_combine_partials) and matches the fp32 reference MoE."""
    from mxserve.ops import moe as moe_mod
    monkeypatch.setattr(moe_mod, "DECODE", True)
    real = moe_mod._fused_experts_decode
    used = []
    monkeypatch.setattr(moe_mod, "_fused_experts_decode", lambda *a: used.append(1) or real(*a))
    H, I, E, K = 512, 1024, 4, 2
    e_local = E if offset == 0 else 2
    g = torch.Generator(device="cuda").manual_seed(T)
    x = torch.randn(T, H, device=gpu, dtype=torch.bfloat16, generator=g)
    w13 = (torch.randn(E, 2 * I, H, device=gpu, generator=g) * 0.05).to(torch.bfloat16)
    w2 = (torch.randn(E, H, I, device=gpu, generator=g) * 0.05).to(torch.bfloat16)
    tw, tid = ops.moe_topk_softmax(torch.randn(T, E, device=gpu, dtype=torch.bfloat16, generator=g), K)
    w13l, w2l = w13[offset:offset + e_local].contiguous(), w2[offset:offset + e_local].contiguous()
    out = moe_mod.fused_experts(x, w13l, w2l, tw, tid, offset)
    assert used and out is not None
    exp = ref.moe_experts(x.cpu(), w13l.cpu(), w2l.cpu(), tw.cpu(), tid.cpu(), offset)
    _close(out, exp, 0.02, 0.03, "moe decode kernel")


def test_moe_experts_uses_grouped_kernel(gpu, monkeypatch):
    from mxserve.ops import moe as moe_mod
    called = []
    monkeypatch.setattr(moe_mod, "_fused_experts_loop", lambda *a, **k: called.append(1))
    H, I, E, K, T = 256, 192, 4, 2, 50
    x = torch.randn(T, H, device=gpu, dtype=torch.bfloat16)
    w13 = torch.randn(E, 2 * I, H, device=gpu, dtype=torch.bfloat16) * 0.05
    w2 = torch.randn(E, H, I, device=gpu, dtype=torch.bfloat16) * 0.05
    tw, tid = ops.moe_topk_softmax(torch.randn(T, E, device=gpu, dtype=torch.bfloat16), K)
    out = moe_mod.fused_experts(x, w13, w2, tw, tid, 2)  # EP: this rank holds experts 2, 3
    assert not called and out is not None
    exp = ref.moe_experts(x.cpu(), w13.cpu(), w2.cpu(), tw.cpu(), tid.cpu(), 2)
    _close(out, exp, 0.02, 0.03, "moe ep")


# ---- serving shapes: the bench runs 4000-token prompts in chunks of up to 8192 tokens and decodes up
# to max_model_len 8192; the fp32 reference runs on the GPU at these sizes
@pytest.mark.parametrize("D,G,hkv", [(64, 4, 2), (128, 4, 1)])
def test_paged_prefill_serving_shape(gpu, D, G, hkv):
    """A 4k cached prefix + an 8k chunk, next to a fresh 1k prompt and a 1-token tail."""
    specs = [(4096, 8192), (0, 1000), (777, 1)]
    seq_lens = [c + n for c, n in specs]
    kv, bt = _paged_setup(seq_lens, hkv, D, device=gpu)
    qsl = [0]
    for _, n in specs:
        qsl.append(qsl[-1] + n)
    q = torch.randn(qsl[-1], hkv * G, D, device=gpu, dtype=torch.bfloat16)
    qsl_t = torch.tensor(qsl, dtype=torch.int32)
    sl = torch.tensor(seq_lens, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    out = ops.paged_attention_prefill(q, kv[:, 1], bt.to(gpu), qsl_t.to(gpu), sl.to(gpu), scale,
                                      max(n for _, n in specs))
    exp = ref.paged_attention(q, kv[:, 1], bt.to(gpu), qsl_t, sl, scale)
    _close(out, exp, 0.03, 0.03, "prefill 4k+8k")


@pytest.mark.parametrize("impl", [1, 2])
@pytest.mark.parametrize("kv_dtype", ["bf16", "fp8"])
@pytest.mark.parametrize("D,G", [(64, 4), (128, 4), (128, 8)])
def test_paged_decode_max_model_len(gpu, D, G, kv_dtype, impl):
    """Contexts up to max_model_len 8192, launched as the decode graphs launch them."""
    hkv, lens = 2, [8192, 8191, 4097, 1, 5000, 16, 6001, 8177]
    kv, bt = _paged_setup(lens, hkv, D, device=gpu)
    ks = vs = 1.0
    if kv_dtype == "fp8":
        ks, vs = 0.02, 0.05
        kv = _fp8_cache(kv * (ks * 4), ks)
    q = torch.randn(len(lens), hkv * G, D, device=gpu, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    out = ops.paged_attention_decode(q, kv[:, 1], bt.to(gpu), sl.to(gpu), scale, 8192, k_scale=ks, v_scale=vs,
                                     impl=impl)
    exp = ref.paged_attention_decode(q, kv[:, 1], bt.to(gpu), sl, scale, ks, vs)
    tol = 0.02 * max(1.0, exp.abs().max().item()) if kv_dtype == "fp8" else 0.02
    _close(out, exp, tol, 0.02, f"decode 8k {kv_dtype}")


@pytest.mark.parametrize("n,e_local,S,k,valid", [(8, 1, 100, 2, 97), (4, 2, 700, 2, 700), (2, 4, 33, 2, 1),
                                                 (8, 1, 2048, 2, 2000)])
def test_ep_route_kernel(gpu, n, e_local, S, k, valid):
    """EP routing on the device: each valid pair's slot is dest * C + (its rank among earlier pairs
    with the same destination) -- a stable, deterministic order --, padding rows get -1, the
    segment ids carry the local expert ids then -1, and the counts match."""
    E = n * e_local
    tid = torch.randint(0, E, (S, k), device=gpu, dtype=torch.int32)
    P, C = S * k, S * k
    slot = torch.empty(P, dtype=torch.int32, device=gpu)
    send_e = torch.full((n * C,), 77, dtype=torch.int32, device=gpu)
    counts = torch.empty(n, dtype=torch.int32, device=gpu)
    ops.ext().ep_route(slot, send_e, counts, tid, valid, e_local, n, C)
    ids = tid.cpu().reshape(-1).tolist()
    exp_slot, exp_e, cnt = [], [-1] * (n * C), [0] * n
    for p, e in enumerate(ids):
        if p // k >= valid:
            exp_slot.append(-1)
            continue
        d = e // e_local
        exp_slot.append(d * C + cnt[d])
        exp_e[d * C + cnt[d]] = e - d * e_local
        cnt[d] += 1
    assert slot.cpu().tolist() == exp_slot
    assert send_e.cpu().tolist() == exp_e
    assert counts.cpu().tolist() == cnt
    rc = torch.empty(n, dtype=torch.int32, device=gpu)
    ops.ext().ep_segment_rows(rc, send_e, C)
    assert rc.cpu().tolist() == cnt
    # rows land at their slots
    hs = torch.randn(S, 64, device=gpu, dtype=torch.bfloat16)
    send_x = torch.zeros(n * C, 64, device=gpu, dtype=torch.bfloat16)
    ops.ext().ep_gather_rows(send_x, hs, slot, k)
    for p in range(0, P, max(1, P // 50)):
        if exp_slot[p] >= 0:
            assert torch.equal(send_x[exp_slot[p]], hs[p // k])


@pytest.mark.parametrize("M,N,K", [(1, 2048, 2048), (100, 3072, 2048), (777, 2048, 8192), (2048, 2048, 2048),
                                   (4096, 3072, 2048), (1000, 16384, 2048)])
def test_prefill_gemm_all_configs(gpu, M, N, K):
    """Prefill projection GEMM kernel (csrc/kernels/gemm_prefill.hip), every tile / split-K
    configuration vs an fp32 reference, including row counts that are not tile multiples."""
    x = (torch.rand(M, K, device=gpu) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=gpu) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    want = x.float() @ w.float().t()
    cfgs = ops.prefill_gemm_configs(M, N, K)
    assert len(cfgs) >= 4
    for cfg in cfgs:
        out = torch.full((M, N), float("nan"), device=gpu, dtype=torch.bfloat16)
        assert ops.prefill_gemm(out, x, w, cfg), cfg
        _close(out, want, atol=2e-2, rtol=2e-2, name=f"prefill gemm {M}x{N}x{K} cfg {cfg}")


def test_prefill_gemm_tuner_and_dispatch(gpu, monkeypatch):
    """Startup tuner for small prefill chunks: hipBLASLt vs the tile kernel per M bucket, and
    ops.linear follows the table (the kernel runs when it was chosen) with correct results."""
    from mxserve.ops import decode_gemm
    monkeypatch.setattr(decode_gemm, "MODE", "auto")
    monkeypatch.setattr(decode_gemm.PREFILL_TABLE, "entries", {})
    w = ((torch.rand(2048, 2048, device=gpu) * 2 - 1) * 0.02).to(torch.bfloat16)
    rows = decode_gemm.tune_prefill({"o": w}, gpu, buckets=(384, 512))
    assert len(rows) == 2 and all(r["us"] <= r["hipblaslt_us"] for r in rows)
    calls = []
    real = ops.prefill_gemm
    monkeypatch.setattr(ops, "prefill_gemm", lambda *a: calls.append(1) or real(*a))
    for M in (300, 500):
        x = torch.randn(M, 2048, device=gpu, dtype=torch.bfloat16)
        _close(ops.linear(x, w), x.float() @ w.float().t(), 2e-2, 2e-2, f"tuned prefill linear M={M}")
    assert len(calls) == sum(r["chosen"] == "mfma" for r in rows)
    x = torch.randn(1000, 2048, device=gpu, dtype=torch.bfloat16)  # above PREFILL_MAX_M: hipBLASLt
    _close(ops.linear(x, w), x.float() @ w.float().t(), 2e-2, 2e-2, "prefill linear M=1000")


def test_sample_top_p_rate(gpu):
    """Top-k / top-p sampling at a serving batch (384 rows x 128k vocab, bf16): the register-resident
    kernel keeps it to a small fraction of a decode step."""
    B, V = 384, 128256
    logits = (torch.randn(B, V, device=gpu) * 3).to(torch.bfloat16)
    t = torch.full((B,), 0.8, device=gpu)
    tp = torch.full((B,), 0.9, device=gpu)
    tk = torch.full((B,), 40, dtype=torch.int32, device=gpu)
    seeds = torch.arange(B, device=gpu)
    steps = torch.zeros(B, dtype=torch.int64, device=gpu)
    ops.sample(logits, t, tp, tk, seeds, steps)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        ops.sample(logits, t, tp, tk, seeds, steps)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print(f"top-k 40 + top-p 0.9 sampling, 384 x 128256 bf16: {ms:.3f} ms")
    assert ms < 2.0


@pytest.mark.parametrize("M,N,K,cfg", [(1, 2048, 2048, (1, 2, 1, 8, 0)), (24, 2048, 8192, (2, 2, 1, 4, 4)),
                                       (256, 2048, 8192, ("mt", 4, 2, 1, 2, 8, 1)),
                                       (200, 2048, 8192, ("mt", 4, 2, 1, 2, 8))])
def test_linear_add_rms_norm_splitk_epilogue(gpu, M, N, K, cfg, monkeypatch):
    """o_proj / down_proj with the split-K slabs summed by the residual-add + RMSNorm epilogue kernel
    (norm_act.hip splitk_add_rmsnorm_kernel) vs the fp32 reference, for the register / LDS decode
    kernels and the mt kernel in both tile orders; the residual is updated in place."""
    from mxserve.ops import decode_gemm
    g = torch.Generator(device="cuda").manual_seed(M + N)
    x = torch.randn(M, K, device=gpu, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=gpu, generator=g) * K ** -0.5).to(torch.bfloat16)
    res = torch.randn(M, N, device=gpu, generator=g).to(torch.bfloat16)
    nw = (1 + 0.1 * torch.randn(N, device=gpu, generator=g)).to(torch.bfloat16)
    y = x.float() @ w.float().t()
    r_want = y.to(torch.bfloat16).float() + res.float()
    h_want = r_want * torch.rsqrt(r_want.pow(2).mean(-1, keepdim=True) + 1e-5) * nw.float()
    tab = decode_gemm.DecodeGemmTable()
    tab.part = torch.empty(8 * M * N, dtype=torch.float32, device=gpu)
    tab.entries[(N, K, 0)] = [(256, cfg)]
    monkeypatch.setattr(decode_gemm, "TABLE", tab)
    monkeypatch.setattr(decode_gemm, "MODE", "auto")
    assert decode_gemm.TABLE.lookup(M, N, K, 0) == cfg
    r = res.clone()
    h, r2 = ops.linear_add_rms_norm(x, w, r, nw, 1e-5)
    assert r2 is r
    _close(r, r_want, atol=3e-2, rtol=2e-2, name=f"residual {cfg}")
    _close(h, h_want, atol=3e-2, rtol=3e-2, name=f"normed {cfg}")
    # the unfused path (hipBLASLt + fused_add_rms_norm) agrees to bf16 rounding
    r3 = res.clone()
    h3, _ = ops.fused_add_rms_norm(torch.nn.functional.linear(x, w), r3, nw, 1e-5)
    _close(h, h3, atol=3e-2, rtol=3e-2, name="fused vs unfused")


@pytest.mark.parametrize("M,cfg,qknorm", [(1, (1, 2, 1, 8, 0), False), (7, (1, 2, 1, 4, 0), True),
                                          (192, ("mt", 4, 2, 1, 2, 4), False), (1, ("sk", 128, 4), False),
                                          (5, ("sk", 128, 4), True), (40, ("sk", 64, 8), False)])
def test_linear_rope_and_cache_splitk(gpu, M, cfg, qknorm, monkeypatch):
    """qkv projection run split-K with its fp32 slabs summed inside the rope / cache-write kernel
    (rope_cache.hip rope_cache_kernel<SLABS>) vs hipBLASLt + the plain rope_and_cache kernel."""
    from mxserve.ops import decode_gemm
    D, hq, hkv, K, nb = 64, 32, 8, 2048, 40
    N = (hq + 2 * hkv) * D
    g = torch.Generator(device="cuda").manual_seed(M)
    h = torch.randn(M, K, device=gpu, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=gpu, generator=g) * K ** -0.5).to(torch.bfloat16)
    cos_sin = ref.build_cos_sin_cache(D, 4096, 500000.0, None, device=gpu)
    pos = torch.randint(0, 4000, (M,), device=gpu, generator=g)
    slots = torch.randperm(nb * 16, device=gpu, generator=g)[:M]
    if M > 2:
        slots[1] = -1  # a padded row: no cache write
    qn = (1 + 0.1 * torch.randn(D, device=gpu, generator=g)).bfloat16() if qknorm else None
    kn = (1 + 0.1 * torch.randn(D, device=gpu, generator=g)).bfloat16() if qknorm else None
    kv = torch.zeros(nb, 2, 2, hkv, 16, D, device=gpu, dtype=torch.bfloat16)
    kv_ref = kv.clone()
    q_ref = ops.rope_and_cache(torch.nn.functional.linear(h, w), hq, hkv, D, pos, cos_sin, kv_ref[:, 1], slots, qn, kn,
                               1e-6)
    tab = decode_gemm.DecodeGemmTable()
    tab.part = torch.empty(8 * M * N, dtype=torch.float32, device=gpu)
    tab.entries[(N, K, 0)] = [(256, cfg)]
    monkeypatch.setattr(decode_gemm, "TABLE", tab)
    monkeypatch.setattr(decode_gemm, "MODE", "auto")
    q = ops.linear_rope_and_cache(h, w, hq, hkv, D, pos, cos_sin, kv[:, 1], slots, qn, kn, 1e-6)
    _close(q, q_ref, 0.03, 0.02, f"q {cfg}")
    _close(kv, kv_ref, 0.03, 0.02, f"kv cache {cfg}")
    assert kv[:, 0].abs().sum().item() == 0


def _strided_q(T, hq, hkv, D, device):
    """q as the attention ops see it on the fused-RoPE path: the first Hq * D columns of qkv rows."""
    qkv = torch.randn(T, (hq + 2 * hkv) * D, device=device, dtype=torch.bfloat16)
    return qkv, qkv[:, :hq * D].view(T, hq, D)


@pytest.mark.parametrize("D,G", [(64, 4), (128, 4), (128, 8), (64, 8)])
@pytest.mark.parametrize("kv_fp8", [False, True])
def test_paged_decode_fused_rope(gpu, D, G, kv_fp8):
    """Decode attention reading un-rotated q from the qkv rows and rotating it in the kernel == the
    reference on the rotated q (the rope kernel's q write skipped)."""
    hkv = 2
    hq = hkv * G
    lens = [513, 2000, 31, 4096, 1]
    kv, bt = _paged_setup(lens, hkv, D, device=gpu)
    B = len(lens)
    _, q = _strided_q(B, hq, hkv, D, gpu)
    pos = torch.tensor([l - 1 for l in lens], device=gpu)
    cos_sin = ref.build_cos_sin_cache(D, 8192, 500000.0, None, device=gpu)
    sl = torch.tensor(lens, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    cache = kv[:, 1]
    sc = {}
    if kv_fp8:
        cache, sc = _fp8_cache(kv[:, 1].contiguous(), 0.05), {"k_scale": 0.05, "v_scale": 0.05}
    out = ops.paged_attention_decode(q, cache, bt.to(gpu), sl.to(gpu), scale, max(lens), rope=(pos, cos_sin), **sc)
    q_rot = ref.apply_rope(q.cpu().float(), pos.cpu(), cos_sin.cpu()).to(torch.bfloat16)
    if kv_fp8:
        exp = ref.paged_attention_decode(q_rot, cache.cpu(), bt, sl, scale, **sc)
    else:
        exp = ref.paged_attention_decode(q_rot, cache.cpu(), bt, sl, scale)
    _close(out, exp, 0.02 * max(1.0, exp.abs().max().item()), 0.02, "decode fused rope")


@pytest.mark.parametrize("var", [None, 128, 256])
@pytest.mark.parametrize("D,G", [(64, 4), (128, 4), (128, 8)])
def test_paged_prefill_fused_rope(gpu, D, G, var):
    """Prefill v3 attention reading un-rotated q from the qkv rows (RoPE applied in the kernel); with
    long prompts the split-KV (128) and paired-tile (256) variants too."""
    hkv = 2
    hq = hkv * G
    specs = [(0, 77), (300, 45), (16, 1), (0, 130), (33, 200)] if var is None else [(0, 1500), (1200, 700), (16, 1)]
    seq_lens = [c + n for c, n in specs]
    kv, bt = _paged_setup(seq_lens, hkv, D, device=gpu)
    qsl = [0]
    for _, n in specs:
        qsl.append(qsl[-1] + n)
    T = qsl[-1]
    _, q = _strided_q(T, hq, hkv, D, gpu)
    pos = torch.cat([torch.arange(c, c + n) for c, n in specs]).to(gpu)
    cos_sin = ref.build_cos_sin_cache(D, 8192, 500000.0, None, device=gpu)
    qsl_t = torch.tensor(qsl, dtype=torch.int32)
    sl = torch.tensor(seq_lens, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    out = ops.paged_attention_prefill(q, kv[:, 1], bt.to(gpu), qsl_t.to(gpu), sl.to(gpu), scale,
                                      max(n for _, n in specs), rope=(pos, cos_sin),
                                      version=0 if var is None else 0x100 + var)
    q_rot = ref.apply_rope(q.cpu().float(), pos.cpu(), cos_sin.cpu()).to(torch.bfloat16)
    exp = ref.paged_attention(q_rot, kv[:, 1].cpu(), bt, qsl_t, sl, scale)
    _close(out, exp, 0.03, 0.03, "prefill fused rope")


@pytest.mark.parametrize("T,D,hkv,slot_kind,kv_fp8", [
    (37, 64, 8, "run", False), (700, 64, 8, "run", False), (4099, 64, 8, "run", False),
    (700, 64, 8, "scrambled", False), (700, 64, 8, "run", True), (1030, 128, 8, "run", False),
    (1030, 128, 1, "scrambled", True), (520, 128, 4, "run", False), (900, 64, 8, "mixed", False),
    (1200, 64, 8, "mixed", True), (2000, 64, 8, "chunks", False)])
def test_rope_kv_only(gpu, T, D, hkv, slot_kind, kv_fp8):
    """rope_and_cache with no q output (the per-token kernel below 512 tokens, kv_rope_t16_kernel at
    and above) writes exactly the K / V the full kernel writes: runs of whole blocks, runs starting
    mid-block, scrambled slots with unmapped (-1) tokens, fp8 caches; "mixed": a mixed step's
    scattered decode rows first (num_decodes: the per-token kernel), then a mid-block prefill run;
    "chunks": several prompts' chunks, each a run through its own non-adjacent blocks."""
    hq = 4 * hkv
    nb = (T + 15) // 16 + 8
    cos_sin = ref.build_cos_sin_cache(D, 8192, 500000.0, None, device=gpu)
    qkv = torch.randn(T, (hq + 2 * hkv) * D, device=gpu, dtype=torch.bfloat16)
    pos = torch.randint(0, 8000, (T,), device=gpu)
    nd = 0
    if slot_kind == "run":
        slots = torch.arange(T, device=gpu) + 16 + (7 if T % 2 else 0)
    elif slot_kind == "mixed":
        nd = 300
        base = (T // 16 + 4) * 16  # decode slots past the prefill run, scattered
        slots = torch.cat([base + torch.randperm(4 * nd, device=gpu)[:nd], torch.arange(T - nd, device=gpu) + 5])
        nb = (base + 4 * nd) // 16 + 1
    elif slot_kind == "chunks":  # 3 prompts: blocks of each drawn from a shuffled pool
        pool = torch.randperm(nb, device=gpu)
        lens, out, bi = [700, 613, T - 1313], [], 0
        for i, L in enumerate(lens):
            start = 9 if i == 1 else 0  # a continuation chunk starting mid-block
            nblk = (start + L + 15) // 16
            blocks = pool[bi:bi + nblk]
            bi += nblk
            pos_in = torch.arange(start, start + L, device=gpu)
            out.append(blocks[pos_in // 16] * 16 + pos_in % 16)
        slots = torch.cat(out)
    else:
        slots = torch.randperm(nb * 16, device=gpu)[:T]
        slots[::13] = -1
    dt = torch.float8_e4m3fn if kv_fp8 else torch.bfloat16
    kv_a = torch.zeros(nb, 2, hkv, 16, D, device=gpu, dtype=torch.bfloat16).to(dt)
    kv_b = kv_a.clone()
    sc = dict(k_scale=0.05, v_scale=0.07) if kv_fp8 else {}
    ops.rope_and_cache(qkv, hq, hkv, D, pos, cos_sin, kv_a, slots, **sc)
    q = ops.rope_kv_into_cache(qkv, hq, hkv, D, pos, cos_sin, kv_b, slots, **sc, num_decodes=nd)
    # V is a copy (bit-exact); K's rotation may contract into FMAs differently per kernel (one rounding
    # step of the stored value at most)
    assert torch.equal(kv_a[:, 1].view(torch.uint8), kv_b[:, 1].view(torch.uint8))
    ka, kb = kv_a[:, 0].float(), kv_b[:, 0].float()
    assert torch.equal(ka == 0, kb == 0), "the same slots written"
    assert (ka - kb).abs().max().item() <= (0.07 if kv_fp8 else 0.02) * ka.abs().max().item()
    assert (ka != kb).float().mean().item() < 0.01
    assert q.data_ptr() == qkv.data_ptr() and q.stride(0) == qkv.shape[1]


@pytest.mark.parametrize("M,N,K,epi", [(4240, 2048, 2048, 0), (4240, 3072, 2048, 0), (4240, 2048, 8192, 0),
                                       (4240, 16384, 2048, 1), (8192, 2048, 2048, 0), (1, 256, 64, 0),
                                       (300, 512, 192, 1), (2048, 4096, 1024, 1), (777, 768, 4096, 0)])
def test_gemm_pf(gpu, M, N, K, epi):
    """Persistent stream-K prefill GEMM (csrc/kernels/gemm_pf.hip) vs fp32: data-parallel rounds,
    stream-K tails (tiles split over workgroups, finished by the head segment), row counts that are not
    tile multiples, SwiGLU epilogue; bitwise repeatable, tile counters left zero."""
    x = (torch.rand(M, K, device=gpu) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=gpu) * 2 - 1) * 2 * K ** -0.5).to(torch.bfloat16)
    w[:, 0] += torch.arange(N, device=gpu, dtype=torch.bfloat16) * 1e-3
    ref = x.float() @ w.float().t()
    if epi == 1:
        ref = torch.nn.functional.silu(ref[:, :N // 2]) * ref[:, N // 2:]
    for tr, mi in [(256, 4), (256, 16), (256, 64), (224, 0), (224, 16), (192, 0), (192, 8), (160, 0), (160, 16), (128, 0), (128, 8)]:
        out = torch.full((M, N // 2 if epi else N), float("nan"), device=gpu, dtype=torch.bfloat16)
        assert ops.gemm_pf(x, w, epi, out, mi, trows=tr) is not None
        _close(out, ref, atol=2e-2, rtol=2e-2, name=f"gemm_pf {M}x{N}x{K} epi{epi} rows {tr} min_iters {mi}")
        again = ops.gemm_pf(x, w, epi, None, mi, trows=tr)
        assert torch.equal(again, out), "stream-K sum must not depend on arrival order"
    slab, cnt, _ = ops._pf_workspace(x.device)
    assert int(cnt.abs().sum()) == 0


@pytest.mark.parametrize("M,N,K", [(4240, 3072, 2048), (6592, 2048, 8192), (777, 2048, 2048)])
def test_hblt_solutions(gpu, M, N, K):
    """hipBLASLt with an explicit solution (csrc/kernels/hblt.cpp) vs fp32: the heuristic's first
    pick and the last supporting solution, plain and r += x W^T in place; an index that names no
    solution is refused (None), not run."""
    x = (torch.rand(M, K, device=gpu) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=gpu) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    r = (torch.rand(M, N, device=gpu) * 2 - 1).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    for resid in (False, True):
        cands = ops.hblt_candidates(M, N, K, resid)
        assert len(cands) > 1
        for sol in (cands[0], cands[-1]):
            if resid:
                rr = r.clone()
                assert ops.hblt_mm(x, w, sol, out=rr, resid=rr) is not None
                _close(rr, ref + r.float(), atol=3e-2, rtol=2e-2, name=f"hblt resid sol {sol}")
            else:
                _close(ops.hblt_mm(x, w, sol), ref, atol=2e-2, rtol=2e-2, name=f"hblt sol {sol}")
    assert ops.hblt_mm(x, w, -12345) is None


def test_hblt_descriptor_cache_eviction(gpu):
    """Prefill row counts differ step to step: hblt.cpp keeps at most 4096 problem descriptors and
    drops them all past that.  Runs across the eviction stay correct (the solution is re-checked
    for every re-created problem)."""
    N, K = 256, 128
    w = (torch.randn(N, K, device=gpu) * 0.1).to(torch.bfloat16)
    xs = (torch.randn(4500, K, device=gpu)).to(torch.bfloat16)
    sol = ops.hblt_candidates(4500, N, K)[0]
    ref = xs.float() @ w.float().t()
    for M in range(257, 257 + 4200):  # 4200 distinct problems: one eviction on the way
        out = ops.hblt_mm(xs[:M], w, sol)
        if out is None:
            continue  # this solution does not take every row count: nothing to check there
        if M % 700 == 0 or M >= 4450:
            _close(out, ref[:M], atol=2e-2, rtol=2e-2, name=f"hblt after {M - 256} problems")
    assert ops.hblt_mm(xs[:300], w, sol) is not None


def test_gemm_pf_fault_word_read_without_sync(gpu):
    """The engine's stats() reads gemm_pf's timeout word through a pinned copy behind the queued work
    (no device sync on the serving loop); once the copy lands it agrees with the synchronous read."""
    x = torch.randn(4240, 2048, device=gpu).to(torch.bfloat16)
    w = (torch.randn(3072, 2048, device=gpu) * 0.02).to(torch.bfloat16)
    assert ops.gemm_pf(x, w, 0, None, 16) is not None
    ops.gemm_pf_faults_async(gpu)  # queues the first copy
    torch.cuda.synchronize()
    assert ops.gemm_pf_faults_async(gpu) == ops.gemm_pf_faults(gpu) == 0


@pytest.mark.parametrize("M,N,K,epi", [(4240, 3072, 2048, 0), (4240, 16384, 2048, 1), (777, 768, 4096, 0),
                                       (300, 512, 192, 1), (6400, 3072, 2048, 0)])
def test_gemm_pf_row_scale(gpu, M, N, K, epi):
    """gemm_pf with the fused-RMSNorm row scale vs fp32 RMSNorm(x, g) @ w.T (SwiGLU after it for epi 1):
    the x^2 sums travel through stream-K slabs, rows past M stay unwritten; the norm weight folded
    into w by ops.fold_norm_weight."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = (torch.randn(M, K, device=gpu, generator=g) * 3).to(torch.bfloat16)
    x[::7] *= 0.01  # rows of very different scale
    nw = (1 + 0.3 * torch.randn(K, device=gpu, generator=g)).to(torch.bfloat16)
    w = (torch.randn(N, K, device=gpu, generator=g) * K ** -0.5).to(torch.bfloat16)
    eps = 1e-5
    xn = x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + eps) * nw.float()
    ref = xn @ w.float().t()
    if epi == 1:
        ref = torch.nn.functional.silu(ref[:, :N // 2]) * ref[:, N // 2:]
    wf = ops.fold_norm_weight(w, nw)
    for mi in (0, 4, 16):
        out = torch.full((M + 3, N // 2 if epi else N), float("nan"), device=gpu, dtype=torch.bfloat16)
        assert ops.gemm_pf(x, wf, epi, out[:M], mi, row_scale=True, eps=eps) is not None
        assert torch.isnan(out[M:].float()).all()
        _close(out[:M], ref, atol=3e-2, rtol=3e-2, name=f"gemm_pf rs {M}x{N}x{K} epi{epi} min_iters {mi}")
        again = ops.gemm_pf(x, wf, epi, None, mi, row_scale=True, eps=eps)
        assert torch.equal(again, out[:M])
    assert int(ops._pf_workspace(x.device)[1].abs().sum()) == 0


@pytest.mark.parametrize("M,N,K", [(4240, 2048, 2048), (4240, 2048, 8192), (777, 768, 4096), (6400, 2048, 8192)])
def test_gemm_pf_residual(gpu, M, N, K):
    """gemm_pf epi 2: out = resid + x @ w.T, in place on the residual stream and out of place."""
    g = torch.Generator(device="cuda").manual_seed(7 * M + N + K)
    x = torch.randn(M, K, device=gpu, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=gpu, generator=g) * K ** -0.5).to(torch.bfloat16)
    r = (torch.randn(M, N, device=gpu, generator=g) * 4).to(torch.bfloat16)
    ref = r.float() + x.float() @ w.float().t()
    for mi, tr in ((0, 256), (16, 256), (0, 224), (8, 160), (0, 128)):
        out = ops.gemm_pf(x, w, 2, None, mi, resid=r, trows=tr)
        _close(out, ref, atol=3e-2, rtol=2e-2, name=f"gemm_pf resid {M}x{N}x{K} mi {mi} rows {tr}")
        rr = r.clone()
        assert ops.gemm_pf(x, w, 2, rr, mi, resid=rr, trows=tr) is not None
        assert torch.equal(rr, out), "in place == out of place"


@pytest.mark.parametrize("M", [1, 5, 16, 17, 32, 40, 64])
@pytest.mark.parametrize("N,K", [(1280, 8192), (8192, 1024), (8192, 3584), (3072, 2048)])
def test_skinny_gemm(gpu, M, N, K):
    """skinny_gemm_kernel (M <= 64 in 1 / 2 / 4 token fragments, 16-column W slices x 4 k-ranges per workgroup) vs an fp32
    reference: bf16 output (one k-group or slabs summed by the reduce kernel) and the raw fp32 slabs
    [groups][M][N] a fused epilogue would read; Llama-3-70B TP-8 shard shapes and the 1B qkv."""
    g = torch.Generator(device="cuda").manual_seed(M * 131 + N + K)
    x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16, generator=g)
    w = (torch.randn(N, K, device=gpu, generator=g) * K ** -0.5).to(torch.bfloat16)
    w[: N // 2] *= 1.5  # asymmetric: a transposed store shows
    want = x.float() @ w.float().t()
    for kr in ((128, 256) if M <= 16 else (64, 128)):
        if K % (4 * kr):
            continue
        groups = K // (4 * kr)
        part = torch.full((groups * M * N,), float("nan"), dtype=torch.float32, device=gpu)
        out = torch.full((M, N), float("nan"), device=gpu, dtype=torch.bfloat16)
        assert ops.ext().skinny_gemm(out, x, w, part, kr, True)
        _close(out, want, atol=2e-2, rtol=2e-2, name=f"skinny {M}x{N}x{K} kr{kr}")
        if groups > 1:
            out2 = torch.full((M, N), float("nan"), device=gpu, dtype=torch.bfloat16)
            assert ops.ext().skinny_gemm(out2, x, w, part, kr, False)
            slabs = part.view(groups, M, N).sum(0)
            _close(slabs, want, atol=2e-2, rtol=2e-2, name=f"skinny slabs {M}x{N}x{K} kr{kr}")
            assert torch.isnan(out2.float()).all(), "reduce=False must leave the output untouched"


@pytest.mark.parametrize("M", [1, 2, 3, 4, 8, 13])
@pytest.mark.parametrize("N,K,epi", [(1280, 8192, 0), (8192, 1024, 0), (8192, 3584, 0), (7168, 8192, 1),
                                     (3072, 2048, 0), (16384, 2048, 1), (2048, 8192, 0)])
def test_gemv_stream(gpu, M, N, K, epi):
    """gemv_stream_kernel (M <= 16, whole W rows streamed, kw waves splitting a workgroup's K, kg
    workgroups splitting K over the grid, SwiGLU in the epilogue or the split-K reduce) at every
    configuration the decode tuner would try, vs an fp32 reference: Llama-3-70B TP-8 shard shapes and the
    1B projections; plus the fp32 result form (kg = 1, epi 0) and the raw slabs (kg > 1, reduce=False)
    the fused epilogues read."""
    from mxserve.ops import decode_gemm
    g = torch.Generator(device="cuda").manual_seed(M * 17 + N + K + epi)
    x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16, generator=g)
    w = (torch.randn(N, K, device=gpu, generator=g) * K ** -0.5).to(torch.bfloat16)
    w[N // 2:] *= 1.5  # halves differ: a swapped gate / up pair or a transposed store shows
    y = x.float() @ w.float().t()
    want = torch.nn.functional.silu(y[:, :N // 2]) * y[:, N // 2:] if epi else y
    cfgs = decode_gemm.gv_candidates(M, N, K, epi)
    assert cfgs or M > 4, "every shape here has a row-stream configuration up to M = 4"
    decode_gemm.TABLE.part = torch.empty(8 * M * N, dtype=torch.float32, device=gpu)
    for cfg in cfgs:
        kg = decode_gemm.DecodeGemmTable.splitk(cfg)
        out = torch.full(want.shape, float("nan"), device=gpu, dtype=torch.bfloat16)
        assert decode_gemm.TABLE.run(out, x, w, cfg, epi), cfg
        _close(out, want, atol=2e-2, rtol=2e-2, name=f"gemv {M}x{N}x{K} epi {epi} {cfg}")
        if not epi and kg == 1:
            part = torch.full((M * N,), float("nan"), dtype=torch.float32, device=gpu)
            assert ops.ext().gemv_stream(out, x, w, part, cfg[1], cfg[2], 0)
            _close(part.view(M, N), want, atol=2e-3, rtol=2e-3, name=f"gemv fp32 {M}x{N}x{K} {cfg}")
        elif not epi:
            part = torch.full((kg * M * N,), float("nan"), dtype=torch.float32, device=gpu)
            out2 = torch.full(want.shape, float("nan"), device=gpu, dtype=torch.bfloat16)
            assert ops.ext().gemv_stream(out2, x, w, part, cfg[1], cfg[2], 0, kg, False)
            _close(part.view(kg, M, N).sum(0), want, atol=2e-3, rtol=2e-3, name=f"gemv slabs {M}x{N}x{K} {cfg}")
            assert torch.isnan(out2.float()).all(), "reduce=False leaves the output untouched"
    assert not ops.ext().gemv_stream(torch.empty(17, want.shape[1], device=gpu, dtype=torch.bfloat16),
                                     torch.zeros(17, K, device=gpu, dtype=torch.bfloat16), w, None, 2, 1, epi), "M <= 16"


@pytest.mark.parametrize("M", [1, 8, 16, 32, 64])
@pytest.mark.parametrize("N,K", [(7168, 8192), (16384, 2048), (2 * 1792, 1024)])
def test_skinny_gemm_swiglu(gpu, M, N, K):
    """skinny_gemm_kernel with the SiLU*mul reduce (epi 1: w = [gate; up], out = SiLU(x gate^T) * (x up^T))
    vs an fp32 reference: Llama-3-70B TP-8 gate_up shard, the 1B gate_up, and a one-k-group shape (the
    single slab still goes through the reduce)."""
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16, generator=g)
    w = (torch.randn(N, K, device=gpu, generator=g) * K ** -0.5).to(torch.bfloat16)
    w[N // 2:] *= 1.5  # gate / up halves differ: a swapped pair shows
    y = x.float() @ w.float().t()
    I = N // 2
    want = torch.nn.functional.silu(y[:, :I]) * y[:, I:]
    for kr in ((128, 256) if M <= 16 else (64, 128)):
        if K % (4 * kr):
            continue
        groups = K // (4 * kr)
        part = torch.full((groups * M * N,), float("nan"), dtype=torch.float32, device=gpu)
        out = torch.full((M, I), float("nan"), device=gpu, dtype=torch.bfloat16)
        assert ops.ext().skinny_gemm(out, x, w, part, kr, True, 1)
        _close(out, want, atol=2e-2, rtol=2e-2, name=f"skinny swiglu {M}x{N}x{K} kr{kr}")
        assert not ops.ext().skinny_gemm(out, x, w, part, kr, False, 1), "SwiGLU needs the reduce"
    from mxserve.ops import decode_gemm
    for cfg in decode_gemm.candidates(M, N, K, 1):
        if cfg[0] == "sk":
            out = torch.full((M, I), float("nan"), device=gpu, dtype=torch.bfloat16)
            decode_gemm.TABLE.part = None
            assert decode_gemm.TABLE.run(out, x, w, cfg, 1), cfg
            _close(out, want, atol=2e-2, rtol=2e-2, name=f"TABLE.run {cfg}")


def _gather_seq_kv(kv_layer, bt_row, L):
    """K, V [L, hkv, D] in fp32 from a paged layer (V blocks are dim-major: ref.gather_kv), on the GPU."""
    k, v = ref.gather_kv(kv_layer, bt_row, L)
    return k.float(), v.float()


def _attn_fp32(q, k, v, qpos, scale):
    """Causal GQA attention in fp32 on the GPU: q [T, Hq, D] at positions qpos over k / v [L, Hkv, D]."""
    T, Hq, D = q.shape
    G = Hq // k.shape[1]
    kk = k.repeat_interleave(G, dim=1).permute(1, 2, 0)  # [Hq, D, L]
    vv = v.repeat_interleave(G, dim=1).permute(1, 0, 2)  # [Hq, L, D]
    s = torch.bmm(q.float().permute(1, 0, 2), kk) * scale  # [Hq, T, L]
    keys = torch.arange(k.shape[0], device=q.device)
    s = s.masked_fill(keys[None, None, :] > qpos[None, :, None], float("-inf"))
    return torch.bmm(torch.softmax(s, dim=-1), vv).permute(1, 0, 2)  # [T, Hq, D]


@pytest.mark.parametrize("var", [None, 0, 128, 256, "v2"])
def test_paged_prefill_long_context(gpu, var):
    """A 1024-token chunk after 64,000 cached tokens (chunked prefill at long context) next to a fresh
    3,000-token prompt, every launch form -- the automatic pick, the explicit default (VAR 0), split-KV
    (128), paired tiles (256) and the v2 kernel -- against fp32 attention over the gathered cache."""
    D, G, hkv = 64, 4, 2
    specs = [(64000, 1024), (0, 3000)]
    seq_lens = [c + n for c, n in specs]
    kv, bt = _paged_setup(seq_lens, hkv, D, L=1, device=gpu)
    qsl = [0]
    for _, n in specs:
        qsl.append(qsl[-1] + n)
    q = torch.randn(qsl[-1], hkv * G, D, device=gpu, dtype=torch.bfloat16)
    scale = 1 / math.sqrt(D)
    out = ops.paged_attention_prefill(q, kv[:, 0], bt.to(gpu), torch.tensor(qsl, dtype=torch.int32, device=gpu),
                                      torch.tensor(seq_lens, dtype=torch.int32, device=gpu), scale,
                                      max(n for _, n in specs),
                                      version=0 if var is None else (2 if var == "v2" else 0x100 + var))
    for i, (c, n) in enumerate(specs):
        k, v = _gather_seq_kv(kv[:, 0], bt[i].to(gpu), c + n)
        exp = _attn_fp32(q[qsl[i]:qsl[i + 1]], k, v, torch.arange(c, c + n, device=gpu), scale)
        _close(out[qsl[i]:qsl[i + 1]], exp, 0.03, 0.03, f"long-context prefill seq {i} var {var}")


def test_paged_decode_long_context(gpu):
    """Decode rows at 131,072 / 70,001 / 17 tokens of context (split-KV partitions + merge) against fp32
    attention over the gathered cache."""
    D, G, hkv = 64, 4, 2
    lens = [131072, 70001, 17]
    kv, bt = _paged_setup(lens, hkv, D, L=1, device=gpu)
    q = torch.randn(len(lens), hkv * G, D, device=gpu, dtype=torch.bfloat16)
    scale = 1 / math.sqrt(D)
    out = ops.paged_attention_decode(q, kv[:, 0], bt.to(gpu), torch.tensor(lens, dtype=torch.int32, device=gpu),
                                     scale, max(lens))
    for i, L in enumerate(lens):
        k, v = _gather_seq_kv(kv[:, 0], bt[i].to(gpu), L)
        exp = _attn_fp32(q[i:i + 1], k, v, torch.tensor([L - 1], device=gpu), scale)
        _close(out[i:i + 1], exp, 0.02, 0.02, f"long-context decode L={L}")


@pytest.mark.parametrize("M,N,K,epi", [(4240, 2048, 2048, 0), (4240, 3072, 2048, 0), (6592, 2048, 8192, 2),
                                       (4240, 16384, 2048, 1), (1, 256, 64, 0), (300, 512, 192, 1),
                                       (777, 768, 4096, 2), (8192, 2048, 2048, 2), (2048, 4096, 1024, 1)])
def test_gemm_w4(gpu, M, N, K, epi):
    """Four-wave prefill GEMM (csrc/kernels/gemm_w4.hip) vs fp32: several tiles per workgroup (the
    k-block stream runs across tiles), partial last token tile, SwiGLU and residual epilogues, the
    residual form in place; bitwise repeatable."""
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K + epi)
    x = (torch.rand(M, K, device=gpu, generator=g) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=gpu, generator=g) * 2 - 1) * 2 * K ** -0.5).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    r = None
    if epi == 1:
        ref = torch.nn.functional.silu(ref[:, :N // 2]) * ref[:, N // 2:]
    elif epi == 2:
        r = (torch.randn(M, N, device=gpu, generator=g) * 2).to(torch.bfloat16)
        ref = ref + r.float()
    out = torch.full((M, N // 2 if epi == 1 else N), float("nan"), device=gpu, dtype=torch.bfloat16)
    assert ops.gemm_w4(x, w, epi, out, resid=r) is not None
    _close(out, ref, atol=3e-2, rtol=2e-2, name=f"gemm_w4 {M}x{N}x{K} epi{epi}")
    again = ops.gemm_w4(x, w, epi, None, resid=r)
    assert torch.equal(again, out)
    if epi == 2:  # in place on the residual stream
        rr = r.clone()
        assert ops.gemm_w4(x, w, 2, rr, resid=rr) is not None
        assert torch.equal(rr, out)

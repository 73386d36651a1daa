"""The attention ops' `rope=` contract on the CPU reference path: un-rotated q (a row-strided view of
the qkv rows, as the fused GPU path passes it) + positions == the reference on pre-rotated q."""
import math

import torch

from mxserve import ops
from mxserve.ops import reference as ref


def _setup(seq_lens, hkv, D, nb_extra=3):
    nbs = [-(-s // 16) for s in seq_lens]
    nb = sum(nbs) + nb_extra
    kv = torch.randn(nb, 2, hkv, 16, D) * 0.5
    bt = torch.zeros(len(seq_lens), max(nbs), dtype=torch.int32)
    o = 0
    for i, n in enumerate(nbs):
        bt[i, :n] = torch.arange(o, o + n, dtype=torch.int32)
        o += n
    return kv, bt


def test_decode_rope_argument_matches_prerotated():
    hq, hkv, D = 8, 2, 64
    lens = [5, 40, 17]
    kv, bt = _setup(lens, hkv, D)
    qkv = torch.randn(len(lens), (hq + 2 * hkv) * D)
    q = qkv[:, :hq * D].view(len(lens), hq, D)
    pos = torch.tensor([l - 1 for l in lens])
    cs = ref.build_cos_sin_cache(D, 128, 10000.0, None)
    sl = torch.tensor(lens, dtype=torch.int32)
    got = ops.paged_attention_decode(q, kv, bt, sl, 1 / math.sqrt(D), max(lens), rope=(pos, cs))
    want = ref.paged_attention_decode(ref.apply_rope(q, pos, cs), kv, bt, sl, 1 / math.sqrt(D))
    assert torch.allclose(got, want, atol=1e-5)


def test_prefill_rope_argument_matches_prerotated():
    hq, hkv, D = 8, 2, 64
    specs = [(0, 9), (20, 7)]
    seq_lens = [c + n for c, n in specs]
    kv, bt = _setup(seq_lens, hkv, D)
    T = sum(n for _, n in specs)
    qkv = torch.randn(T, (hq + 2 * hkv) * D)
    q = qkv[:, :hq * D].view(T, hq, D)
    pos = torch.cat([torch.arange(c, c + n) for c, n in specs])
    cs = ref.build_cos_sin_cache(D, 128, 10000.0, None)
    qsl = torch.tensor([0, 9, 16], dtype=torch.int32)
    sl = torch.tensor(seq_lens, dtype=torch.int32)
    got = ops.paged_attention_prefill(q, kv, bt, qsl, sl, 1 / math.sqrt(D), 9, rope=(pos, cs))
    want = ref.paged_attention(ref.apply_rope(q, pos, cs), kv, bt, qsl, sl, 1 / math.sqrt(D))
    assert torch.allclose(got, want, atol=1e-5)

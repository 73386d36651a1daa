"""Which prefill-attention variant a launch picks (csrc/kernels/attention_prefill.hip pf3_effective_var),
checked on the host: the selection is pure arithmetic on the launch shape, no GPU involved.

D = 64 has 512 resident workgroups (2 per CU), D = 128 256: split-KV (128) when the unsplit grid is at
most 640 / 320 workgroups, paired q-tiles (256) when the paired grid fills the resident workgroups at
least once, else the default (0).  Explicit versions (0x100 + VAR) pass through; the v2 kernel (-1)
only for version 2 on a bf16 cache with a dense q."""
import pytest

from mxserve import ops

pytestmark = pytest.mark.skipif(not ops.has_ext(), reason="native extension not built")


def pick(num_seqs, max_q_len, D=64, hq=32, hkv=8, version=3, fp8=False, fused_q=True):
    return ops.ext().paged_prefill_variant(version, fp8, fused_q, num_seqs, max_q_len, hq, hkv, D)


@pytest.mark.parametrize("shape,want", [
    ((1, 1024), 128), ((1, 2048), 128), ((1, 4096), 128),  # <= 640 q-tile workgroups: split
    ((2, 4096), 256), ((4, 2048), 256), ((8, 1024), 256), ((1, 8192), 256), ((2, 8192), 256),  # paired grid >= 512
    ((1, 6144), 0), ((2, 3000), 0), ((3, 2000), 0),  # in between: neither pays
])
def test_d64_selection(shape, want):
    assert pick(*shape) == want


@pytest.mark.parametrize("shape,want", [((1, 2048), 128), ((2, 4096), 256), ((1, 8192), 256), ((1, 3000), 0)])
def test_d128_selection(shape, want):
    assert pick(*shape, D=128) == want


def test_fp8_cache_and_gqa_use_the_same_gate():
    assert pick(2, 4096, fp8=True) == 256
    assert pick(1, 2048, fp8=True) == 128
    # G = 1 (32 kv heads): 256-token tiles, 4x the kv heads of G = 4
    assert pick(1, 4096, hq=32, hkv=32) == 128  # 16 tiles x 32 heads = 512 workgroups
    assert pick(1, 8192, hq=32, hkv=32) == 256  # 32 x 32 = 1024; paired 512


def test_explicit_versions():
    assert pick(1, 8192, version=0x100 + 128) == 128
    assert pick(1, 1024, version=0x100 + 256) == 256
    assert pick(1, 1024, version=0x100 + 2) == 2  # softmax variants: bf16 cache, G = 4
    assert pick(1, 1024, version=0x100 + 2, fp8=True) == 0
    assert pick(1, 1024, version=0x100 + 2, hq=16, hkv=8) == 0


def test_v2_only_for_bf16_dense_q():
    assert pick(1, 4096, version=2, fused_q=False) == -1
    assert pick(1, 4096, version=2, fused_q=True) == 128  # fused q needs v3
    assert pick(1, 4096, version=2, fp8=True, fused_q=False) == 128


@pytest.mark.parametrize("version", [2, 3])
@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("fused_q", [False, True])
@pytest.mark.parametrize("shape", [(1, 2048), (2, 4096), (1, 6144)])
def test_split_scratch_matches_the_reported_variant(version, fp8, fused_q, shape):
    """the split scratch / counters are sized from the same v2-vs-v3 decision the launch and
    the variant report use -- version 2 with a fused q runs v3, so its split variant gets scratch."""
    var = pick(*shape, version=version, fp8=fp8, fused_q=fused_q)
    ws, cnt = ops.ext().paged_prefill_split_need(version, fp8, fused_q, shape[0], shape[1], 32, 8, 64)
    assert (ws > 0 and cnt > 0) == (var == 128), (var, ws, cnt)

"""Row-chunk planner of the paired-tile bf16 Gram (ops/gram.pair_chunks): pure host
arithmetic, so it is pinned on the CPU. The kernel's results do not depend on the plan
beyond fp32 partial-sum order (tests/test_gpu.py checks the Gram values on a GPU)."""
import pytest

from ate_replication_causalml_amd.ops.gram import pair_chunks


def _check(seg_bounds, K, chunks, seg_chunk0):
    assert seg_chunk0[0] == 0 and seg_chunk0[-1] == len(chunks)
    for s, (r0, r1) in enumerate(seg_bounds):
        cs = chunks[seg_chunk0[s]:seg_chunk0[s + 1]]
        assert cs, "every segment gets at least one chunk"
        assert cs[0][0] == r0 and cs[-1][1] == r1
        for (a, e, seg, _), nxt in zip(cs, cs[1:] + [None]):
            assert seg == s and a <= e
            if nxt is not None:
                assert e == nxt[0] and (e - a) % K == 0   # contiguous, whole K-steps
        lens = [e - a for a, e, _, _ in cs[:-1]]
        if lens:
            assert max(lens) - min(lens) <= K              # near-equal


@pytest.mark.parametrize("nseg,rows,target,ncu,want", [
    (5, 2_000_000, 1280, 256, 1280),    # the bench shape: 5 whole rounds on 256 CUs
    (5, 2_000_000, 2048, 0, 2040),      # explicit target: 2 x 5 x 204
    (5, 2_000_000, 2048, 256, 1280),    # rounded down to whole rounds (k 204 -> 128)
    (10, 1_000_000, 1280, 256, 1280),
    (3, 3_000_000, 1280, 256, 768),
    (1, 10_000_000, 1280, 256, 1280),
])
def test_pair_chunks_counts(nseg, rows, target, ncu, want):
    segs = [(s * rows, (s + 1) * rows) for s in range(nseg)]
    chunks, c0 = pair_chunks(segs, 64, 2, target, ncu)
    assert 2 * len(chunks) == want
    _check(segs, 64, chunks, c0)


def test_pair_chunks_small_segments():
    # panels pad every segment to a positive multiple of 64 rows (ops/panel.py ROW_ALIGN)
    segs = [(0, 64), (64, 64 + 64 * 5), (384, 384 + 128)]
    chunks, c0 = pair_chunks(segs, 64, 2, 2048, 256)
    _check(segs, 64, chunks, c0)
    # a segment shorter than its chunk count gets one chunk per K-step
    assert [c0[s + 1] - c0[s] for s in range(3)] == [1, 5, 2]


def test_tri_blocks_cover_the_upper_triangle_once():
    """Split-triangle kernel (P == 512): the slab table names every 16-column block I <= J of
    the 32 x 32 block triangle exactly once; the type-0 workgroup only blocks of the first 22
    columns blocks (the 352 columns it stages), every wave at most 36 blocks."""
    from ate_replication_causalml_amd.ops.gram import TRI_SLOTS, TRI_SPLIT, tri_blocks, tri_roles
    tb = tri_blocks()
    assert len(tb) == 2 and all(len(t) == TRI_SLOTS for t in tb)
    used = [b for t in tb for b in t if b[0] >= 0]
    assert sorted(used) == [(i, j) for i in range(32) for j in range(i, 32)]
    assert all(j < TRI_SPLIT for i, j in tb[0] if i >= 0)
    for roles in tri_roles():
        assert len(roles) == 8
        for fc, bl in roles:
            assert len(bl) <= 36 and len(set(fc)) == len(fc)
            assert all(fc[a] <= fc[b] for a, b in bl)


@pytest.mark.parametrize("nt", [2, 3, 4])
@pytest.mark.parametrize("bal", [True, False])
def test_pair_tiles_cover_the_upper_triangle_once(nt, bal):
    """Paired-tile slab table (csrc/gram.hip gram_bf16_pair_kernel): every 16-column block
    I <= J once, for the balanced (34 / 34 blocks per diagonal-pair wave, GRAM_BAL) and the
    unbalanced (32 / 36) wave roles."""
    from ate_replication_causalml_amd.ops.gram import PAIR_SLOTS, _pair_tiles
    tiles, blocks = _pair_tiles(nt, bal)
    assert all(len(t) == PAIR_SLOTS for t in blocks)
    used = [b for t in blocks for b in t if b[0] >= 0]
    assert sorted(used) == [(i, j) for i in range(16 * nt) for j in range(i, 16 * nt)]

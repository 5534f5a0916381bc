"""The backward's LDS bank layout (lgm_amd/csrc/render_raster.hip, k_render_bwd), restated on the host: the lane
groups and bank functions of MI355X's LDS instructions (ds_write_b32: banks (a/4) mod 32 in two 32-lane groups;
ds_read_b128: banks (a/4) mod 64, four non-contiguous 16-lane groups) applied to the kernel's address formulas.
Checks that (1) a batch's moment stores put the 32 lanes of each group on 32 distinct banks whenever the batch's
8 entry columns are consecutive, and (2) the batch reads of the swizzled w / u image put each 16-lane group on 16
distinct 16-B slots. Pure host arithmetic (no GPU); it mirrors the constants of the kernel, so a change there that
breaks the layout has to change this test too."""
from collections import Counter

CH, MB, NC = 64, 8, 3  # BWD_CHUNK, entries per batch, colour channels (no depth gradient)
NROW = 6 + 2 * NC
LS = CH + 4
JB = (LS * NROW + 31) & ~31
WU_LD = 68
B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128_GROUPS += [[x + 32 for x in g] for g in B128_GROUPS]


def mrow(lane, rr):
    """k_render_bwd's per-lane slot offset of MFMA result rr (the moment row, or a junk offset)."""
    ql, qk = lane & 15, lane >> 4

    def is_live(qq, ucol):
        row = 4 * qq + rr
        return (6 <= row < NROW) if ucol else row <= 5
    ucol = ql >= MB
    live = is_live(qk, ucol)
    m = 2 * (qk & 1) + (0 if live else (1 if (is_live(qk, not ucol) or ucol) else 0))
    return 4 * qk * LS + rr * LS if live else JB + ((rr * LS + 8 * m) & 31)


def wu_swz(col):
    return 8 if 4 <= col < 12 else 0


def test_moment_stores_are_conflict_free_for_consecutive_columns():
    assert LS % 32 == 4
    for c0 in range(0, CH - MB + 1):
        cols = [c0 + (lane & 7) for lane in range(64)]  # the lane's batch column (ql & 7) -> entry
        for rr in range(4):
            addr = [mrow(lane, rr) + cols[lane] for lane in range(64)]
            for half in (range(0, 32), range(32, 64)):
                banks = Counter(addr[lane] % 32 for lane in half)
                assert max(banks.values()) == 1, (c0, rr, banks.most_common(2))
            live = [a for a in addr if a < LS * NROW]
            assert len(set(live)) == len(live)  # two live results never share a slot word
            assert all(a < JB + 32 + CH + 4 for a in addr)  # inside the slot


def test_live_moment_rows_match_the_features():
    # w columns keep the 6 geometric moments (rows 0..5), u columns the colour hi / lo sums (rows 6..NROW-1)
    kept = {(lane & 15, 4 * (lane >> 4) + rr) for lane in range(64) for rr in range(4) if mrow(lane, rr) < JB}
    assert kept == {(ql, row) for ql in range(16) for row in range(NROW) if (row <= 5) == (ql < MB)}


def test_batch_reads_of_the_swizzled_image_are_conflict_free():
    for t2 in range(2):
        for h in range(2):
            for g in B128_GROUPS:
                slots = []
                for lane in g:
                    ql, qk = lane & 15, lane >> 4
                    p = (32 * t2 + 8 * qk + 4 * h) ^ wu_swz(ql)
                    slots.append(((ql * WU_LD + p) // 4) % 16)
                assert len(set(slots)) == 16, (t2, h, g[:4])


def test_swizzled_writes_stay_a_permutation():
    # each image row is written as pixel lane -> lane ^ wu_swz(column): a permutation of the row's 64 words, so the
    # 32 lanes of each ds_write2_b32 group still hit 32 distinct banks
    for col in range(16):
        pos = [lane ^ wu_swz(col) for lane in range(64)]
        assert sorted(pos) == list(range(64))
        for half in (range(0, 32), range(32, 64)):
            assert len({(col * WU_LD + pos[lane]) % 32 for lane in half}) == 32

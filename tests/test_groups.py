"""EnvGroups' env ranges (host logic; the GPU equivalence is tests/test_gpu_groups.py)."""

import pytest

from zbot_amd.engine import ZbError, group_bounds


@pytest.mark.parametrize("n,G", [(8192, 2), (8192, 4), (517, 2), (300, 3), (64, 4), (5, 5), (3, 2), (7, 3), (1, 1)])
def test_bounds_cover_every_env_once(n, G):
    b = group_bounds(n, G)
    assert len(b) == G
    assert b[0][0] == 0 and b[-1][1] == n
    assert all(lo < hi for lo, hi in b)
    assert all(b[i][1] == b[i + 1][0] for i in range(G - 1))
    sizes = [hi - lo for lo, hi in b]
    assert max(sizes) - min(sizes) <= 2


def test_bounds_on_whole_pairs_when_possible():
    assert group_bounds(8192, 2) == [(0, 4096), (4096, 8192)]
    assert all(lo % 2 == 0 for lo, _ in group_bounds(517, 2))
    assert all(lo % 2 == 0 for lo, _ in group_bounds(32768, 4))


@pytest.mark.parametrize("n,G", [(4, 0), (2, 3)])
def test_bad_group_counts_raise(n, G):
    with pytest.raises(ZbError):
        group_bounds(n, G)

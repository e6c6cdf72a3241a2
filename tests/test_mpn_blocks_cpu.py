"""Host logic of the MPN's per-call size split (mpn/model.py::node_blocks): contiguous node blocks that no
edge crosses, packed greedily under the edge and node limits of one libpemp call."""
import pytest
import torch

from oracle import restate
from pemp_amd.mpn.model import node_blocks


def _batch(sizes, isolated=0):
    parts, off = [], 0
    for n in sizes:
        parts.append(restate.fully_edge_index(n) + off)
        off += n
    return torch.cat(parts, 1), off + isolated


def test_blocks_pack_images_greedily():
    ei, N = _batch([5, 4, 6])                       # 20, 12, 30 edges
    assert node_blocks(ei, N, 30, 100) == [(0, 5), (5, 9), (9, 15)]
    assert node_blocks(ei, N, 32, 100) == [(0, 9), (9, 15)]
    assert node_blocks(ei, N, 1000, 9) == [(0, 9), (9, 15)]
    assert node_blocks(ei, N, 1000, 1000) == [(0, 15)]


def test_blocks_never_cut_an_edge():
    g = torch.Generator().manual_seed(3)
    ei, N = _batch([7, 1, 9, 3, 12, 2], isolated=3)
    ei = ei[:, torch.randperm(ei.shape[1], generator=g)]    # any edge order; both directions present
    for lim in (132, 140, 204, 300):
        blocks = node_blocks(ei, N, lim, 1 << 20)
        assert blocks[0][0] == 0 and blocks[-1][1] == N
        assert all(a[1] == b[0] for a, b in zip(blocks, blocks[1:]))
        blk = torch.zeros(N, dtype=torch.long)
        for k, (n0, n1) in enumerate(blocks):
            blk[n0:n1] = k
        assert torch.equal(blk[ei[0]], blk[ei[1]])
        assert max(int(((blk[ei[0]] == k)).sum()) for k in range(len(blocks))) <= lim


def test_blocks_refuse_an_indivisible_block():
    ei, N = _batch([5, 6])
    with pytest.raises(NotImplementedError):
        node_blocks(ei, N, 25, 100)                 # the 6-node image alone has 30 edges
    with pytest.raises(ValueError):
        node_blocks(ei, N - 1, 1000, 1000)          # node id out of range


def test_blocks_without_edges():
    assert node_blocks(torch.zeros(2, 0, dtype=torch.long), 3, 1, 1) == [(0, 1), (1, 2), (2, 3)]
    assert node_blocks(torch.zeros(2, 0, dtype=torch.long), 0, 1, 1) == []


@pytest.mark.parametrize("rows,n,L", [(3, 3, 7), (1, 0, 5), (4, 4, 1), (2, 2, 0), (5, 3, 2)])
def test_logit_rows_match_view_squeeze(rows, n, L):
    """mpn/model.py::_rows (one unbind) returns what the reference's per-row view(L, 1).squeeze() returns: same
    shapes (a 0-d tensor for L == 1), values, strides and storage."""
    from pemp_amd.mpn.model import _rows
    buf = torch.arange(rows * L, dtype=torch.float32).view(rows, L)
    got = _rows(buf, n)
    ref = [buf[r].view(L, 1).squeeze() for r in range(n)]
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        assert a.shape == b.shape and a.stride() == b.stride() and a.data_ptr() == b.data_ptr()
        assert torch.equal(a, b)

"""CPU: the peer all-reduce's work partition (csrc/peer_kernels.hip, PeerPartition) covers every
element of a bucket exactly once, in 16-byte-aligned pieces, for any count / world size /
block count -- the property the kernel's per-block flag protocol relies on."""
from hypothesis import given, settings
from hypothesis import strategies as st


def _native():
    import mxddp

    return mxddp.native()


def _pieces(count, ws, blocks, vec):
    chunk, sl = _native().PeerComm.partition(count, ws, blocks, vec)
    out = []
    for p in range(ws):
        for b in range(blocks):
            lo = b * sl
            hi = min(lo + sl, chunk)
            n = max(0, min(count - p * chunk, hi) - lo)
            if n:
                out.append((p * chunk + lo, n))
    return chunk, sl, out


@settings(max_examples=300, deadline=None)
@given(count=st.integers(1, 3_000_000), ws=st.integers(2, 8), blocks=st.sampled_from([1, 7, 16, 64, 256]),
       vec=st.sampled_from([4, 8]))
def test_partition_covers_exactly_once(count, ws, blocks, vec):
    chunk, sl, pieces = _pieces(count, ws, blocks, vec)
    assert chunk % vec == 0 and sl % vec == 0
    assert chunk * ws >= count
    pieces.sort()
    pos = 0
    for start, n in pieces:
        assert start == pos, (start, pos)
        assert start % vec == 0  # 16-byte aligned vector start
        pos += n
    assert pos == count


def test_mnist_bucket_partition():
    # the fused engine's fc bucket (4.72 MB) over 8 ranks and 64 blocks
    chunk, sl, pieces = _pieces(1_181_066, 8, 64, 4)
    assert chunk == 147_636 and sl == 2_308
    assert sum(n for _, n in pieces) == 1_181_066

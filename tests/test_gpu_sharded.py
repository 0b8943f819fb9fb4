"""mqvs_sharded_search (libmqvs's own RCCL communicator) on the GPU box's one
GPU: a 1-rank communicator runs the whole exchange path -- chunk-count
all-gather (cosine), local search, (id, distance) all-gather, device merge --
and must equal mqvs_search bit for bit.  The multi-rank decomposition (shard
ranges, ordinal bases, merge order) is covered on CPU with gloo
(tests/test_sharded.py); N > 1 GPUs run in the driver's scaling bench."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    import myscaledb_amd as m
    from myscaledb_amd.sharded import RcclComm
    m.init(0)
    c = RcclComm(1, 0, RcclComm.unique_id())
    yield c
    c.free()


@pytest.mark.parametrize("metric,nq,k,filt", [("Cosine", 24, 50, None), ("L2", 3, 20, 0.3), ("IP", 40, 100, None),
                                              ("Cosine", 2, 30, 0.2), ("L2", 20, 5000, None)])
def test_one_rank_sharded_search_equals_search(comm, metric, nq, k, filt):
    import myscaledb_amd as mq
    n, d, gran = 30000, 48, 1024
    rows = O.generate(101, 1, 0, n, d)
    q = O.generate(102, 1, 0, nq, d)
    rng = np.random.default_rng(4)
    flt = mq.pack_bitmap(rng.random(n) < filt) if filt else None
    rex = mq.pack_bitmap(rng.random(n) >= 0.1)
    seg = mq.VectorScanSegment.from_rows(rows, metric=metric, granule=gran)
    try:
        a = seg.search(q, k, filter_bitmap=flt, row_exists=rex)
        b = comm.sharded_search(seg, q, k, filter_bitmap=flt, row_exists=rex)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))
        import torch
        tq = torch.from_numpy(q).cuda()
        ti, td = comm.sharded_search(seg, tq, k, filter_bitmap=None if flt is None else torch.from_numpy(flt).cuda(),
                                     row_exists=torch.from_numpy(rex).cuda())
        assert np.array_equal(ti.cpu().numpy(), a[0])
        assert np.array_equal(td.cpu().numpy().view(np.uint32), a[1].view(np.uint32))
    finally:
        seg.free()


def test_comm_errors(comm):
    from myscaledb_amd._lib import MqvsError
    from myscaledb_amd.sharded import RcclComm
    with pytest.raises(MqvsError):
        RcclComm(2, 5, bytes(128))

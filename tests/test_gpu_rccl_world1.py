"""bench.py --gpus N's process set-up, rehearsed on the one GPU (VERDICT r05
item 6): torch.distributed's "nccl" group (RCCL) and libmqvs's own dlopen'ed
RCCL communicator live in ONE process -- torch's group is created first and
carries a collective, then RcclComm.from_process_group() builds libmqvs's
communicator from it (the unique id would travel by a broadcast over the
group at N > 1) and mqvs_sharded_search runs several times: the first call on
the validated path, the next ones on the one-sync fast path (its counter
advances), every result bit-identical to mqvs_search.  This is the sequence
bench.py runs under torch.distributed.run (bench.py main: init_process_group
("nccl"), RcclComm.from_process_group, rank_main); it replaces the
Distributed engine's per-shard LIMIT + initiator merge
(StorageDistributed.cpp:1057-1060) and the cross-part merge
(MergeTreeBaseSearchManager.cpp:207-297)."""
import os
import socket

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_torch_nccl_group_then_rccl_comm_sharded_search():
    import torch
    import torch.distributed as dist
    import myscaledb_amd as mq
    from myscaledb_amd.sharded import RcclComm
    torch.cuda.set_device(0)
    assert not dist.is_initialized()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    comm = seg = None
    try:
        mq.init(0)
        # torch's RCCL communicator exists and works before libmqvs's
        t = torch.ones(4, device="cuda")
        dist.all_reduce(t)
        assert t.sum().item() == 4
        comm = RcclComm.from_process_group()
        assert (comm.nranks, comm.rank) == (1, 0)
        n, d, gran = 50000, 64, 2048
        seg = mq.VectorScanSegment.from_rows(O.generate(201, 2, 0, n, d), metric="Cosine", granule=gran)
        cases = [(O.generate(202, 2, 0, 8, d), 30), (O.generate(203, 2, 0, 300, d), 100)]
        for q, k in cases:
            exp = seg.search(q, k)
            tq = torch.from_numpy(q).cuda()
            for rep in range(3):
                ids, dist_ = comm.sharded_search(seg, tq, k)
                torch.cuda.synchronize()
                assert np.array_equal(ids.cpu().numpy(), exp[0]), rep
                assert np.array_equal(dist_.cpu().numpy().view(np.uint32), exp[1].view(np.uint32)), rep
            hi, hd = comm.sharded_search(seg, q, k)  # host pointers: a different call, validated again
            assert np.array_equal(hi, exp[0]) and np.array_equal(hd.view(np.uint32), exp[1].view(np.uint32))
        st = comm.stats()
        # per case: 1 validated + 2 fast device calls, then 1 validated host call
        assert st["fast_calls"] == 4 and st["redo_calls"] == 0, st
        # torch's group still works after libmqvs's collectives
        t2 = torch.full((8,), 2.0, device="cuda")
        dist.all_reduce(t2)
        assert t2.sum().item() == 16
    finally:
        if comm is not None:
            comm.free()
        if seg is not None:
            seg.free()
        dist.destroy_process_group()

"""Re-entrancy (the reference admits 2 x physical cores
concurrent scans, MergeTreeVSManager.cpp:974-975): many host threads search
the same resident segments at once -- each thread gets its own HIP stream and
workspace, there is no global lock -- and every result equals the sequential
one bit for bit.  ctypes releases the GIL around each C call, so the searches
really overlap."""
import threading

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mq():
    import myscaledb_amd as m
    m.init(0)
    return m


def test_concurrent_searches_match_sequential(mq):
    n, d, gran = 60000, 96, 4096
    segs = {
        "L2": mq.VectorScanSegment.from_rows(O.generate(1, 1, 0, n, d), metric="L2", granule=gran),
        "Cosine": mq.VectorScanSegment.from_rows(O.generate(2, 2, 0, n, d), metric="Cosine", granule=gran),
    }
    rng = np.random.default_rng(0)
    # a mix of batch sizes that exercises every path (VALU, bf16 pre-filter)
    jobs = []
    for i in range(48):
        metric = "L2" if i % 2 else "Cosine"
        nq = [1, 3, 8, 19, 25, 64, 150][i % 7]
        k = [10, 50, 100][i % 3]
        q = O.generate(100 + i, 1, 0, nq, d)
        flt = mq.pack_bitmap(rng.random(n) > 0.3) if i % 5 == 0 else None
        jobs.append((metric, q, k, flt))
    expected = [segs[m].search(q, k, filter_bitmap=f) for m, q, k, f in jobs]

    results = [None] * len(jobs)
    errors = []

    def worker(tid, nthreads):
        try:
            mq.init(0)
            for rep in range(2):
                for j in range(tid, len(jobs), nthreads):
                    m, q, k, f = jobs[j]
                    results[j] = segs[m].search(q, k, filter_bitmap=f)
            from myscaledb_amd import _lib
            _lib.check(_lib.lib.mqvs_thread_release())
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    threads = [threading.Thread(target=worker, args=(t, 16)) for t in range(16)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert not errors, errors
    for j, ((ie, de), got) in enumerate(zip(expected, results)):
        assert got is not None, j
        ig, dg = got
        assert np.array_equal(ig, ie), j
        assert np.array_equal(dg.view(np.uint32), de.view(np.uint32)), j
    for s in segs.values():
        s.free()

"""The reference-side C++ binding (include/mqvs_vector_index.hpp) compiled with
g++ against libmqvs.so, as a MyScaleDB maintainer would use it
(INTEGRATION.md).  CPU: status -> DB::Exception code mapping, including
tryBruteForceSearch's NOT_IMPLEMENTED for non-float metrics
(BruteForceSearch.h:89).  GPU: tryBruteForceSearch / PartScan::scan / rerank
through the shim vs the oracle; k = 8000 (PartScan::search), the 1-rank RCCL
ShardComm, GpuIndex (search / computeTopDistanceSubset / setRowIdsMap),
getRealBitmap and the PartCache (load / pin / evict / forceExpire)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def shim_bin(tmp_path_factory):
    out = tmp_path_factory.mktemp("shim") / "shim_check"
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-DMQVS_SHIM_STANDALONE",
           "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests/shim/shim_check.cpp"),
           "-L", os.path.join(ROOT, "myscaledb_amd"), "-l:libmqvs.so",
           "-Wl,-rpath," + os.path.join(ROOT, "myscaledb_amd"), "-Wl,-rpath,/opt/rocm/lib",
           "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return str(out)


def test_shim_compiles_and_maps_errors(shim_bin):
    r = subprocess.run([shim_bin, "errors"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "errors ok" in r.stdout


def test_shim_device_failure_falls_back(shim_bin):
    """on a device error the host runs its CPU path.  An injected
    failure (mqvs_inject_fault: MQVS_ERR_DEVICE, then MQVS_ERR_MEMORY_LIMIT)
    makes tryBruteForceSearch run the caller's fallback -- the faiss call of
    BruteForceSearch.h:80-87 in the ClickHouse tree -- and return its result;
    without a fallback the status is rethrown with its DB::ErrorCodes value,
    and other statuses (NOT_IMPLEMENTED) never fall back."""
    r = subprocess.run([shim_bin, "fallback"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "fallback ok" in r.stdout


def _val(i, j):
    return np.float32(((i * 31 + j * 17) % 23) - 11)


@pytest.mark.gpu
def test_shim_gpu_matches_oracle(shim_bin, tmp_path):
    from oracle import oracle as O
    r = subprocess.run([shim_bin, "gpu", str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "rerank==search 1" in r.stdout
    n, d, nq, k, gran = 3000, 24, 5, 12, 512
    i, j = np.meshgrid(np.arange(n), np.arange(d), indexing="ij")
    rows = (((i * 31 + j * 17) % 23) - 11).astype(np.float32)
    i, j = np.meshgrid(np.arange(nq) + 7777, np.arange(d), indexing="ij")
    q = ((((i * 31 + j * 17) % 23) - 11).astype(np.float32) * np.float32(0.5)).astype(np.float32)

    def rd(name, dt):
        return np.fromfile(tmp_path / name, dtype=dt)

    for m, tag in ((O.L2, "l2"), (O.IP, "ip")):
        io, do = O.knn(q, rows, k, m)
        assert np.array_equal(rd(f"knn_{tag}_ids.bin", np.int64).reshape(nq, k), io), tag
        assert np.array_equal(rd(f"knn_{tag}_dist.bin", np.float32).reshape(nq, k).view(np.uint32),
                              do.view(np.uint32)), tag
    io, do = O.vector_scan(rows, q, k, O.COSINE, gran)
    keep = io.reshape(-1) > -1
    assert np.array_equal(rd("scan_label.bin", np.uint32), io.reshape(-1)[keep].astype(np.uint32))
    assert np.array_equal(rd("scan_vid.bin", np.uint32),
                          (np.arange(nq * k) // k)[keep].astype(np.uint32))
    assert np.array_equal(rd("scan_dist.bin", np.float32).view(np.uint32),
                          do.reshape(-1)[keep].view(np.uint32))
    for tag in ("sharded==search 1", "gpu fallback 1", "row_ids_map 1", "getRealBitmap 1", "cache 1", "prefilter active 1"):
        assert tag in r.stdout, r.stdout
    # k = 8000 over the 12000-row L2 part == the oracle's vectorScanWithoutIndex
    nl, kl = 12000, 8000
    i, j = np.meshgrid(np.arange(nl) + 3, np.arange(d), indexing="ij")
    lrows = (((i * 31 + j * 17) % 23) - 11).astype(np.float32)
    io, do = O.vector_scan(lrows, q, kl, O.L2, gran)
    assert np.array_equal(rd("bigk_ids.bin", np.int64).reshape(nq, kl), io)
    assert np.array_equal(rd("bigk_dist.bin", np.float32).reshape(nq, kl).view(np.uint32), do.view(np.uint32))
    # two-stage index search: the re-ranked distances are the exact ones of the
    # first stage's rows (oracle knn over those rows), best first
    fs = rd("index_fs_ids.bin", np.int64).reshape(nq, 64)
    ri = rd("index_rerank_ids.bin", np.int64).reshape(nq, 12)
    rdist = rd("index_rerank_dist.bin", np.float32).reshape(nq, 12)
    for qi in range(nq):
        cand = fs[qi][fs[qi] >= 0]
        ki, kd = O.knn(q[qi:qi + 1], lrows[cand], 12, O.L2)
        assert np.array_equal(ri[qi], cand[ki[0]]), qi
        assert np.array_equal(rdist[qi].view(np.uint32), kd[0].view(np.uint32)), qi

// Timing of the cosine query prep (k_query_prep, kernels_misc.hip) on the
// bench's query distributions: nq queries of generator mode m (held-out rows
// n .. n + nq, as tools/index_sweep.py draws them), maxv 12; prints the kernel
// time and the histogram of mu + lambda (normalisations to the first repeat).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off tools/qprep_probe.hip -o tools/bin/qprep_probe
#include "../myscaledb_amd/csrc/kernels_misc.hip"

#include <cstdio>
#include <map>
#include <vector>

using namespace mqvs;

int main() {
    const int nq = 1000, d = 768, maxv = 12;
    const int64_t n = 10000000;
    float *q, *qv, *qn;
    int *mu, *lam, *st;
    (void)hipMalloc(&q, sizeof(float) * nq * d);
    (void)hipMalloc(&qv, sizeof(float) * (size_t)nq * maxv * d);
    (void)hipMalloc(&qn, sizeof(float) * nq);
    (void)hipMalloc(&mu, sizeof(int) * nq);
    (void)hipMalloc(&lam, sizeof(int) * nq);
    (void)hipMalloc(&st, sizeof(int) * 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int mode = 0; mode < 4; ++mode) {
        launch_generate(0x5EED0001ull, mode, n, nq, d, q, 0);
        float best = 1e9f;
        for (int it = 0; it < 5; ++it) {
            (void)hipMemset(st, 0, 16);
            (void)hipEventRecord(a);
            launch_query_prep(q, nq, d, MQVS_METRIC_COSINE, false, qv, maxv, qn, mu, lam, st, 0);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        std::vector<int> hm(nq), hl(nq);
        (void)hipMemcpy(hm.data(), mu, sizeof(int) * nq, hipMemcpyDeviceToHost);
        (void)hipMemcpy(hl.data(), lam, sizeof(int) * nq, hipMemcpyDeviceToHost);
        std::map<int, int> h;
        for (int i = 0; i < nq; ++i) h[hm[i] + hl[i]]++;
        printf("mode %d: %.1f us; mu+lambda:", mode, best * 1e3);
        for (auto &kv : h) printf(" %d:%d", kv.first, kv.second);
        printf("\n");
    }
    return 0;
}

// A/B of the cosine query prep's sequential square sum (kernels_misc.hip
// k_query_prep): SUMV 0 = v_readlane walk, 1 = LDS broadcast walk, 2 = the
// LDS walk software-pipelined, 3 = register phases (seq_sq_sum_lanes).  All must write bit-identical variant tables;
// prints the best of 20 launches at nq = 1 and nq = 1000 (generator mode 1,
// d = 768, maxv 32), and the floor of a 768-long dependent add chain from
// registers (chain_us: one wave, `reps` chains, no loads) for scale.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off tools/qprep_sum_ab.hip -o tools/bin/qprep_sum_ab
#include "../myscaledb_amd/csrc/kernels_misc.hip"

#include <cstdio>
#include <cstring>
#include <vector>

using namespace mqvs;

__global__ void k_chain(const float *in, float *out, int reps) {
    float x[12];
#pragma unroll
    for (int u = 0; u < 12; ++u) x[u] = in[threadIdx.x + 64 * u];
    float acc = 0.f;
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int i = 0; i < 64; ++i)
#pragma unroll
            for (int u = 0; u < 12; ++u) acc = acc + x[u];
    }
    out[threadIdx.x] = acc;
}

static float chain_us(const float *in, float *out, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e9f;
    for (int it = 0; it < 20; ++it) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, in, out, reps);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    return best * 1e3f;
}

template <int V, bool LS = false>
static float run(const float *q, int nq, int d, int maxv, float *qv, float *qn, int *mu, int *lam, int *st) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e9f;
    const size_t sig = LS ? (size_t)(maxv + 1) * 64 * sizeof(uint32_t) : (size_t)(maxv + 1) * sizeof(uint64_t);
    for (int it = 0; it < 20; ++it) {
        (void)hipMemset(st, 0, 16);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL((k_query_prep<12, V, LS>), dim3(nq), dim3(64), sig, 0, q, nq, d, MQVS_METRIC_COSINE, 0, qv, maxv,
                           qn, mu, lam, st, 0);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    return best * 1e3f;
}

int main() {
    const int d = 768, maxv = 32;
    for (int nq : {1, 1000}) {
        float *q, *qv[5], *qn;
        int *mu, *lam, *st;
        (void)hipMalloc(&q, sizeof(float) * nq * d);
        for (auto &p : qv) (void)hipMalloc(&p, sizeof(float) * (size_t)nq * maxv * d);
        (void)hipMalloc(&qn, sizeof(float) * nq);
        (void)hipMalloc(&mu, sizeof(int) * nq);
        (void)hipMalloc(&lam, sizeof(int) * nq);
        (void)hipMalloc(&st, sizeof(int) * 4);
        launch_generate(0x5EED0002ull, 1, 0, nq, d, q, 0);
        const float t0 = run<0>(q, nq, d, maxv, qv[0], qn, mu, lam, st);
        const float t1 = run<1>(q, nq, d, maxv, qv[1], qn, mu, lam, st);
        const float t2 = run<2>(q, nq, d, maxv, qv[2], qn, mu, lam, st);
        const float t3 = run<3>(q, nq, d, maxv, qv[3], qn, mu, lam, st);
        const float t4 = run<3, true>(q, nq, d, maxv, qv[4], qn, mu, lam, st);
        std::vector<float> h0((size_t)nq * maxv * d), h1(h0.size()), h2(h0.size()), h3(h0.size()), h4(h0.size());
        (void)hipMemcpy(h0.data(), qv[0], h0.size() * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(h1.data(), qv[1], h1.size() * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(h2.data(), qv[2], h2.size() * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(h3.data(), qv[3], h3.size() * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(h4.data(), qv[4], h4.size() * 4, hipMemcpyDeviceToHost);
        const bool same = std::memcmp(h0.data(), h1.data(), h0.size() * 4) == 0 &&
                          std::memcmp(h0.data(), h2.data(), h0.size() * 4) == 0 &&
                          std::memcmp(h0.data(), h3.data(), h0.size() * 4) == 0 &&
                          std::memcmp(h0.data(), h4.data(), h0.size() * 4) == 0;
        int hmu = 0, hlam = 0;
        (void)hipMemcpy(&hmu, mu, 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&hlam, lam, 4, hipMemcpyDeviceToHost);
        std::printf("{\"nq\": %d, \"readlane_us\": %.2f, \"lds_us\": %.2f, \"lds_pipe_us\": %.2f, "
                    "\"lanes_us\": %.2f, \"lanes_lanesig_us\": %.2f, \"bitwise_equal\": %s, \"q0_mu\": %d, \"q0_lam\": %d}\n",
                    nq, t0, t1, t2, t3, t4, same ? "true" : "false", hmu, hlam);
        if (nq == 1) {
            float *cout;
            (void)hipMalloc(&cout, sizeof(float) * 64);
            const float c1 = chain_us(q, cout, 1), c9 = chain_us(q, cout, 9);
            std::printf("{\"chain_768_us\": %.3f, \"launch_plus_one_chain_us\": %.2f, \"nine_chains_us\": %.2f}\n",
                        (c9 - c1) / 8.0f, c1, c9);
        }
    }
    return 0;
}

// Microbenchmark of the sequential fp32 sum of squares (k_query_prep's chain,
// kernels_misc.hip): readlane walk vs LDS float4 walk, 1000 waves x R
// normalisations of a 768-vector.  Checks both give the same bits.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/seqsum_probe.hip -o /tmp/seqsum && /tmp/seqsum
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

constexpr int J = 12;

__device__ __forceinline__ float sum_readlane(const float (&x)[J]) {
    float acc = 0.0f;
#pragma unroll
    for (int u = 0; u < J; ++u) {
        const int sq = __builtin_bit_cast(int, x[u] * x[u]);
#pragma unroll
        for (int l0 = 0; l0 < 64; l0 += 16) {
            float t[16];
#pragma unroll
            for (int l = 0; l < 16; ++l) t[l] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(sq, l0 + l));
#pragma unroll
            for (int l = 0; l < 16; ++l) acc = acc + t[l];
        }
    }
    return acc;
}

__device__ __forceinline__ float sum_lds(const float (&x)[J], float *sb) {
    const int lane = threadIdx.x;
#pragma unroll
    for (int u = 0; u < J; ++u) sb[lane + 64 * u] = x[u] * x[u];
    __syncthreads();
    const float4 *s4 = reinterpret_cast<const float4 *>(sb);
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 16 * J; ++k) {
        const float4 a = s4[k];
        acc = acc + a.x;
        acc = acc + a.y;
        acc = acc + a.z;
        acc = acc + a.w;
    }
    __syncthreads();
    return acc;
}

template <int MODE>
__global__ __launch_bounds__(64) void k_norm(const float *q, int R, float *out) {
    __shared__ __attribute__((aligned(16))) float sb[64 * J];
    const int lane = threadIdx.x;
    float x[J];
#pragma unroll
    for (int u = 0; u < J; ++u) x[u] = q[blockIdx.x * 64 * J + lane + 64 * u];
    float last = 0.f;
    for (int r = 0; r < R; ++r) {
        const float s = MODE == 0 ? sum_readlane(x) : sum_lds(x, sb);
        const float sr = sqrtf(s);
#pragma unroll
        for (int u = 0; u < J; ++u) x[u] = x[u] / sr;
        last = s;
    }
    if (lane == 0) out[blockIdx.x] = last;
#pragma unroll
    for (int u = 0; u < J; ++u) out[gridDim.x + blockIdx.x * 64 * J + lane + 64 * u] = x[u];
}

int main() {
    const int nq = 1000, R = 13;
    std::vector<float> h((size_t)nq * 64 * J);
    unsigned s = 1;
    for (auto &v : h) {
        s = s * 1664525u + 1013904223u;
        v = ((s >> 8) / 16777216.0f - 0.5f) * 3.0f;
    }
    float *dq, *o0, *o1;
    hipMalloc(&dq, h.size() * 4);
    hipMalloc(&o0, (nq + h.size()) * 4);
    hipMalloc(&o1, (nq + h.size()) * 4);
    hipMemcpy(dq, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int mode = 0; mode < 2; ++mode) {
        float best = 1e9f;
        for (int it = 0; it < 10; ++it) {
            hipEventRecord(a);
            if (mode == 0)
                hipLaunchKernelGGL(k_norm<0>, dim3(nq), dim3(64), 0, 0, dq, R, o0);
            else
                hipLaunchKernelGGL(k_norm<1>, dim3(nq), dim3(64), 0, 0, dq, R, o1);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        printf("mode %d (%s): %.1f us for %d normalisations\n", mode, mode ? "lds float4" : "readlane", best * 1e3, R);
    }
    std::vector<float> r0(nq + h.size()), r1(nq + h.size());
    hipMemcpy(r0.data(), o0, r0.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(r1.data(), o1, r1.size() * 4, hipMemcpyDeviceToHost);
    printf("bitwise equal: %s\n", memcmp(r0.data(), r1.data(), r0.size() * 4) == 0 ? "yes" : "NO");
    return 0;
}

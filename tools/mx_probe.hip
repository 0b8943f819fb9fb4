// mx_probe.hip -- hardware facts for the block-scaled (MX) MFMA on gfx950,
// measured rather than assumed (tools only, not part of the library):
//   1. operand layout of v_mfma_scale_f32_32x32x64_f8f6f4 with fp6 e2m3 and
//      fp8 e4m3 operands: which lane/bit holds A[i][k] / B[k][j], which lane's
//      scale applies to which block -- checked against a CPU product of random
//      codes and random E8M0 scales (exact: every partial sum is a short dyadic)
//   2. issue rate of the bf16, fp8-MX and fp6-MX forms (cycles per MFMA per
//      SIMD from a dependent-free loop over 4 accumulators).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mx_probe.hip -o gpurun_out/mx_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

static double e2m3_val(int code) {
    const int s = (code >> 5) & 1, e = (code >> 3) & 3, m = code & 7;
    const double v = e == 0 ? m / 8.0 : std::ldexp(1.0 + m / 8.0, e - 1);
    return s ? -v : v;
}
static double e4m3_val(int code) {
    const int s = (code >> 7) & 1, e = (code >> 3) & 15, m = code & 7;
    if (e == 15 && m == 7) return NAN;
    const double v = e == 0 ? std::ldexp(m / 8.0, -6) : std::ldexp(1.0 + m / 8.0, e - 7);
    return s ? -v : v;
}

// FMT 2 = fp6 e2m3 (6 VGPRs, element j at bits 6j), 0 = fp8 e4m3 (8 VGPRs, byte j)
template <int FMT>
__global__ void k_layout(const v8i *a, const v8i *b, const int *sa, const int *sb, float *out) {
    const int l = threadIdx.x;
    f32x16 c = {0};
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[l], b[l], c, FMT, FMT, 0, sa[l], 0, sb[l]);
    for (int r = 0; r < 16; ++r) out[l * 16 + r] = c[r];
}

template <int FMT>
static int layout_test(unsigned seed) {
    std::srand(seed);
    const int bits = FMT == 2 ? 6 : 8;
    int A[32][64], B[64][32], SA[64], SB[64];
    for (int i = 0; i < 32; ++i)
        for (int k = 0; k < 64; ++k) A[i][k] = std::rand() & ((1 << bits) - 1);
    for (int k = 0; k < 64; ++k)
        for (int j = 0; j < 32; ++j) B[k][j] = std::rand() & ((1 << bits) - 1);
    if (FMT == 0) {  // no NaN codes
        for (auto &r : A)
            for (int &v : r)
                if ((v & 0x7f) == 0x7f) v &= 0xfe;
        for (auto &r : B)
            for (int &v : r)
                if ((v & 0x7f) == 0x7f) v &= 0xfe;
    }
    for (int l = 0; l < 64; ++l) {
        SA[l] = 124 + std::rand() % 7;
        SB[l] = 124 + std::rand() % 7;
    }
    // hypothesis: lane l holds A[l & 31][32 (l >> 5) + j] and B[32 (l >> 5) + j][l & 31]
    // as element j; its scale applies to those 32 elements
    std::vector<v8i> ha(64), hb(64);
    for (int l = 0; l < 64; ++l) {
        uint32_t wa[8] = {0}, wb[8] = {0};
        for (int j = 0; j < 32; ++j) {
            const int ca = A[l & 31][32 * (l >> 5) + j], cb = B[32 * (l >> 5) + j][l & 31];
            const int bit = j * bits;
            wa[bit / 32] |= (uint32_t)ca << (bit % 32);
            wb[bit / 32] |= (uint32_t)cb << (bit % 32);
            if (bit % 32 + bits > 32) {
                wa[bit / 32 + 1] |= (uint32_t)ca >> (32 - bit % 32);
                wb[bit / 32 + 1] |= (uint32_t)cb >> (32 - bit % 32);
            }
        }
        for (int w = 0; w < 8; ++w) {
            ha[l][w] = (int)wa[w];
            hb[l][w] = (int)wb[w];
        }
    }
    v8i *da, *db;
    int *dsa, *dsb;
    float *dout;
    CK(hipMalloc(&da, 64 * sizeof(v8i)));
    CK(hipMalloc(&db, 64 * sizeof(v8i)));
    CK(hipMalloc(&dsa, 64 * 4));
    CK(hipMalloc(&dsb, 64 * 4));
    CK(hipMalloc(&dout, 64 * 16 * 4));
    CK(hipMemcpy(da, ha.data(), 64 * sizeof(v8i), hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), 64 * sizeof(v8i), hipMemcpyHostToDevice));
    CK(hipMemcpy(dsa, SA, 64 * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsb, SB, 64 * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_layout<FMT>, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dout);
    CK(hipDeviceSynchronize());
    float out[64 * 16];
    CK(hipMemcpy(out, dout, sizeof(out), hipMemcpyDeviceToHost));
    int bad = 0;
    double maxrel = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) {
            const int col = l & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
            double ref = 0;
            for (int k = 0; k < 64; ++k) {
                const int h = k >> 5;
                const double va = (FMT == 2 ? e2m3_val(A[row][k]) : e4m3_val(A[row][k])) *
                                  std::ldexp(1.0, SA[row + 32 * h] - 127);
                const double vb = (FMT == 2 ? e2m3_val(B[k][col]) : e4m3_val(B[k][col])) *
                                  std::ldexp(1.0, SB[col + 32 * h] - 127);
                ref += va * vb;
            }
            const double g = out[l * 16 + r];
            const double rel = std::fabs(g - ref) / (std::fabs(ref) + 1e-30);
            if (rel > maxrel) maxrel = rel;
            if (rel > 1e-6) {
                if (bad < 4) std::printf("  fmt %d mismatch row %d col %d: gpu %.9g ref %.9g\n", FMT, row, col, g, ref);
                ++bad;
            }
        }
    std::printf("layout fmt=%d (%s): %d / 1024 mismatches, max rel err %.3g\n", FMT, FMT == 2 ? "fp6 e2m3" : "fp8 e4m3",
                bad, maxrel);
    CK(hipFree(da));
    CK(hipFree(db));
    CK(hipFree(dsa));
    CK(hipFree(dsb));
    CK(hipFree(dout));
    return bad;
}

// throughput: KIND 0 bf16 32x32x16, 1 fp8-MX 32x32x64, 2 fp6-MX 32x32x64,
// 3 bf16 16x16x32, 4 fp6-MX 16x16x128
template <int KIND>
__global__ __launch_bounds__(256) void k_rate(float *sink, int iters, int seed) {
    v8i a, b;
    for (int i = 0; i < 8; ++i) {
        a[i] = 0x01020304 * (threadIdx.x + i + seed) & 0x1f1f1f1f;
        b[i] = 0x04030201 * (threadIdx.x + 2 * i + seed) & 0x1f1f1f1f;
    }
    bf16x8 ab, bb;
    for (int i = 0; i < 8; ++i) {
        ab[i] = (__bf16)(float)(threadIdx.x + i);
        bb[i] = (__bf16)(float)(i - (int)threadIdx.x);
    }
    f32x16 c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
    f32x4 d0 = {0}, d1 = {0}, d2 = {0}, d3 = {0};
    for (int it = 0; it < iters; ++it) {
        if (KIND == 0) {
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, c3, 0, 0, 0);
        } else if (KIND == 1 || KIND == 2) {
            constexpr int F = KIND == 1 ? 0 : 2;
            c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c0, F, F, 0, 127, 0, 127);
            c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c1, F, F, 0, 127, 0, 127);
            c2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c2, F, F, 0, 127, 0, 127);
            c3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c3, F, F, 0, 127, 0, 127);
        } else if (KIND == 3) {
            d0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, d0, 0, 0, 0);
            d1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, d1, 0, 0, 0);
            d2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, d2, 0, 0, 0);
            d3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, d3, 0, 0, 0);
        } else {
            d0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, d0, 2, 2, 0, 127, 0, 127);
            d1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, d1, 2, 2, 0, 127, 0, 127);
            d2 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, d2, 2, 2, 0, 127, 0, 127);
            d3 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, d3, 2, 2, 0, 127, 0, 127);
        }
    }
    float s = 0;
    for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
    for (int r = 0; r < 4; ++r) s += d0[r] + d1[r] + d2[r] + d3[r];
    if (s == 1.2345f) sink[threadIdx.x] = s;
}

template <int KIND>
static void rate(const char *name, double flops_per_mfma) {
    float *sink;
    CK(hipMalloc(&sink, 1024 * 4));
    const int iters = 20000, blocks = 256 * 8;  // 8 waves/CU x 4 waves/block... 2 blocks per SIMD-group
    hipLaunchKernelGGL(k_rate<KIND>, dim3(blocks), dim3(256), 0, 0, sink, 100, 1);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_rate<KIND>, dim3(blocks), dim3(256), 0, 0, sink, iters, 2);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double n = (double)blocks * 4 /*waves*/ * iters * 4 /*mfma*/;
    const double tf = n * flops_per_mfma / (ms * 1e-3) / 1e12;
    // cycles per MFMA per SIMD at the measured rate, assuming 2.4 GHz, 1024 SIMDs
    const double cyc = (ms * 1e-3) * 2.4e9 * 1024 / n;
    std::printf("rate %-22s %8.3f ms  %8.1f TF/s (dense-equivalent)  ~%.1f cycles/MFMA/SIMD @2.4GHz\n", name, ms, tf,
                cyc);
    CK(hipFree(sink));
}

int main() {
    int bad = 0;
    bad += layout_test<2>(1);
    bad += layout_test<2>(7);
    bad += layout_test<0>(3);
    rate<0>("bf16 32x32x16", 2.0 * 32 * 32 * 16);
    rate<3>("bf16 16x16x32", 2.0 * 16 * 16 * 32);
    rate<1>("fp8-MX 32x32x64", 2.0 * 32 * 32 * 64);
    rate<2>("fp6-MX 32x32x64", 2.0 * 32 * 32 * 64);
    rate<4>("fp6-MX 16x16x128", 2.0 * 16 * 16 * 128);
    return bad ? 1 : 0;
}

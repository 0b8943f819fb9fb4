// mfma_acc_probe.hip -- the accumulation error of the MFMA forms the
// pre-filters bound, measured against exact sums (tools only, not part of the
// library).  The pre-filter bounds (kernels_bf16.hip k_query_bound) assume:
//   bf16 (v_mfma_f32_32x32x16_bf16, chained over K = d): products are exact in
//     fp32 and every addition errs by at most 2u of the running |sum| (u =
//     2^-24; 2u covers round-toward-zero), so |err| <= 2.04 d u sum|a_k b_k|;
//   fp6-MX (v_mfma_scale_f32_32x32x64_f8f6f4, e2m3 x e2m3 with E8M0 block
//     scales, chained): |err| <= 2^-10 sum|a_k b_k| (the "MX internal"
//     allowance) + the same 2u-per-addition chain term.
// For each case this prints the worst ratio err / (u sum|a_k b_k|) over the
// 32 x 32 outputs; the bounds hold when the bf16 ratio stays <= 2.04 d and the
// MX ratio <= 2^14 + 3.03 d (2^-10 / u = 2^14).  Exact reference: long double
// sums of exact products (bf16 and scaled e2m3 values and their products are
// dyadic with few significant bits).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_acc_probe.hip -o gpurun_out/mfma_acc_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            std::exit(1);                                                                         \
        }                                                                                         \
    } while (0)

constexpr int K = 768;  // the headline dimension: 48 bf16 MFMAs / 12 MX MFMAs chained

// A [32][K], B [K][32] as bf16 bit patterns; lane l feeds A[l & 31][16 s + 8 (l >> 5) + e]
// and B[16 s + 8 (l >> 5) + e][l & 31] at step s (the layout kernels_hi.hip reads)
__global__ void k_bf16(const uint16_t *A, const uint16_t *B, float *out) {
    const int l = threadIdx.x;
    f32x16 c = {0};
    for (int s = 0; s < K / 16; ++s) {
        bf16x8 a, b;
        for (int e = 0; e < 8; ++e) {
            const int k = 16 * s + 8 * (l >> 5) + e;
            a[e] = __builtin_bit_cast(__bf16, A[(l & 31) * K + k]);
            b[e] = __builtin_bit_cast(__bf16, B[k * 32 + (l & 31)]);
        }
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
    for (int r = 0; r < 16; ++r) out[l * 16 + r] = c[r];
}

// fp6 e2m3 codes A [32][K], B [K][32]; scales (E8M0) SA [K/32][32] (per row and
// 32-block), SB [K/32][32] (per column and block).  Lane l at step s holds
// A[l & 31][64 s + 32 (l >> 5) + j], j < 32 (mx_probe.hip's measured layout).
__global__ void k_mx(const uint8_t *A, const uint8_t *B, const int *SA, const int *SB, float *out) {
    const int l = threadIdx.x;
    f32x16 c = {0};
    for (int s = 0; s < K / 64; ++s) {
        uint32_t wa[8] = {0}, wb[8] = {0};
        for (int j = 0; j < 32; ++j) {
            const int k = 64 * s + 32 * (l >> 5) + j;
            const uint32_t ca = A[(l & 31) * K + k], cb = B[k * 32 + (l & 31)];
            const int bit = 6 * j;
            wa[bit / 32] |= ca << (bit % 32);
            wb[bit / 32] |= cb << (bit % 32);
            if (bit % 32 + 6 > 32) {
                wa[bit / 32 + 1] |= ca >> (32 - bit % 32);
                wb[bit / 32 + 1] |= cb >> (32 - bit % 32);
            }
        }
        v8i a, b;
        for (int w = 0; w < 8; ++w) {
            a[w] = (int)wa[w];
            b[w] = (int)wb[w];
        }
        const int blk = 2 * s + (l >> 5);
        c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 2, 2, 0, SA[blk * 32 + (l & 31)], 0,
                                                             SB[blk * 32 + (l & 31)]);
    }
    for (int r = 0; r < 16; ++r) out[l * 16 + r] = c[r];
}

static uint16_t to_bf16(float x) {  // round to nearest even
    uint32_t u;
    std::memcpy(&u, &x, 4);
    u += 0x7fff + ((u >> 16) & 1);
    return (uint16_t)(u >> 16);
}
static long double bf16_val(uint16_t h) {
    const uint32_t u = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
static long double e2m3_val(int code) {
    const int s = (code >> 5) & 1, e = (code >> 3) & 3, m = code & 7;
    const long double v = e == 0 ? m / 8.0L : std::ldexp(1.0L + m / 8.0L, e - 1);
    return s ? -v : v;
}

static void run_bf16(const char *name, const std::vector<float> &a, const std::vector<float> &b, double &worst) {
    std::vector<uint16_t> A(32 * K), B(K * 32);
    for (int i = 0; i < 32 * K; ++i) A[i] = to_bf16(a[i]);
    for (int i = 0; i < K * 32; ++i) B[i] = to_bf16(b[i]);
    uint16_t *dA, *dB;
    float *dO;
    CK(hipMalloc(&dA, A.size() * 2));
    CK(hipMalloc(&dB, B.size() * 2));
    CK(hipMalloc(&dO, 64 * 16 * 4));
    CK(hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_bf16, dim3(1), dim3(64), 0, 0, dA, dB, dO);
    CK(hipDeviceSynchronize());
    float out[64 * 16];
    CK(hipMemcpy(out, dO, sizeof(out), hipMemcpyDeviceToHost));
    double mr = 0, mrel = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) {
            const int col = l & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
            long double ref = 0, mag = 0;
            for (int k = 0; k < K; ++k) {
                const long double p = bf16_val(A[row * K + k]) * bf16_val(B[k * 32 + col]);
                ref += p;
                mag += fabsl(p);
            }
            const double err = (double)fabsl((long double)out[l * 16 + r] - ref);
            const double ratio = mag > 0 ? err / ((double)mag * 5.9604644775390625e-8) : 0.0;
            if (ratio > mr) mr = ratio;
            if (mag > 0 && err / (double)mag > mrel) mrel = err / (double)mag;
        }
    if (mr > worst) worst = mr;
    std::printf("bf16  %-34s max err/(u sum|p|) = %10.3f   max err/sum|p| = %.3g   (bound 2.04 d = %.0f)\n", name, mr,
                mrel, 2.04 * K);
    CK(hipFree(dA));
    CK(hipFree(dB));
    CK(hipFree(dO));
}

static void run_mx(const char *name, const std::vector<uint8_t> &A, const std::vector<uint8_t> &B,
                   const std::vector<int> &SA, const std::vector<int> &SB, double &worst) {
    uint8_t *dA, *dB;
    int *dSA, *dSB;
    float *dO;
    CK(hipMalloc(&dA, A.size()));
    CK(hipMalloc(&dB, B.size()));
    CK(hipMalloc(&dSA, SA.size() * 4));
    CK(hipMalloc(&dSB, SB.size() * 4));
    CK(hipMalloc(&dO, 64 * 16 * 4));
    CK(hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dSA, SA.data(), SA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dSB, SB.data(), SB.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_mx, dim3(1), dim3(64), 0, 0, dA, dB, dSA, dSB, dO);
    CK(hipDeviceSynchronize());
    float out[64 * 16];
    CK(hipMemcpy(out, dO, sizeof(out), hipMemcpyDeviceToHost));
    double mr = 0, mrel = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) {
            const int col = l & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
            long double ref = 0, mag = 0;
            for (int k = 0; k < K; ++k) {
                const int blk = k / 32;
                const long double va = e2m3_val(A[row * K + k]) * std::ldexp(1.0L, SA[blk * 32 + row] - 127);
                const long double vb = e2m3_val(B[k * 32 + col]) * std::ldexp(1.0L, SB[blk * 32 + col] - 127);
                ref += va * vb;
                mag += fabsl(va * vb);
            }
            const double err = (double)fabsl((long double)out[l * 16 + r] - ref);
            const double ratio = mag > 0 ? err / ((double)mag * 5.9604644775390625e-8) : 0.0;
            if (ratio > mr) mr = ratio;
            if (mag > 0 && err / (double)mag > mrel) mrel = err / (double)mag;
        }
    if (mr > worst) worst = mr;
    std::printf("fp6MX %-34s max err/(u sum|p|) = %10.3f   max err/sum|p| = %.3g   (allowance 2^-10 + 3.03 d u: "
                "ratio %.0f)\n",
                name, mr, mrel, 16384.0 + 3.03 * K);
    CK(hipFree(dA));
    CK(hipFree(dB));
    CK(hipFree(dSA));
    CK(hipFree(dSB));
    CK(hipFree(dO));
}

int main() {
    std::mt19937_64 g(12345);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::uniform_int_distribution<int> ui(0, 1 << 30);
    double wb = 0, wm = 0;
    std::vector<float> a(32 * K), b(K * 32);

    // ---- bf16 ----
    for (auto &v : a) v = nd(g);
    for (auto &v : b) v = nd(g);
    run_bf16("gaussian", a, b, wb);
    for (auto &v : a) v = std::fabs(nd(g)) + 1.f;
    for (auto &v : b) v = std::fabs(nd(g)) + 1.f;
    run_bf16("all positive (growing partial sums)", a, b, wb);
    for (int i = 0; i < 32; ++i)
        for (int k = 0; k < K; ++k) {
            a[i * K + k] = (k & 1) ? -1024.f * (1.f + (k % 7) / 8.f) : 1024.f * (1.f + ((k - 1 + 7) % 7) / 8.f);
            if (k % 5 == 0) a[i * K + k] = std::ldexp(1.f + (i % 8) / 8.f, -12);
        }
    for (auto &v : b) v = 1.f;
    run_bf16("cancellation (+-2^10 pairs, 2^-12 terms)", a, b, wb);
    for (auto &v : a) v = std::ldexp(1.f + (ui(g) % 128) / 128.f, (ui(g) % 41) - 20);
    for (auto &v : b) v = std::ldexp((ui(g) & 1 ? -1.f : 1.f) * (1.f + (ui(g) % 128) / 128.f), (ui(g) % 41) - 20);
    run_bf16("exponents 2^-20..2^20, mixed signs", a, b, wb);
    for (int i = 0; i < 32; ++i)
        for (int k = 0; k < K; ++k) a[i * K + k] = k == 0 ? 1.f : std::ldexp(1.f - 1.f / 256.f, -25 - (i % 4));
    for (auto &v : b) v = 1.f;
    run_bf16("1 + many terms just under half an ulp", a, b, wb);
    for (int i = 0; i < 32; ++i)
        for (int k = 0; k < K; ++k) a[i * K + k] = k == 0 ? 1.f : std::ldexp(1.f - 1.f / 256.f, -24);
    run_bf16("1 + many terms just under one ulp", a, b, wb);

    // ---- fp6 MX ----
    std::vector<uint8_t> A(32 * K), B(K * 32);
    std::vector<int> SA(K / 32 * 32), SB(K / 32 * 32);
    auto rnd_codes = [&](std::vector<uint8_t> &v) {
        for (auto &c : v) c = ui(g) & 63;
    };
    rnd_codes(A);
    rnd_codes(B);
    for (auto &s : SA) s = 127;
    for (auto &s : SB) s = 127;
    run_mx("random codes, unit scales", A, B, SA, SB, wm);
    for (auto &s : SA) s = 107 + ui(g) % 41;
    for (auto &s : SB) s = 107 + ui(g) % 41;
    run_mx("random codes, scales 2^-20..2^20", A, B, SA, SB, wm);
    for (auto &c : A) c = 0x1f;  // +7.5, the largest e2m3 magnitude
    for (auto &c : B) c = 0x1f;
    for (auto &s : SA) s = 127;
    for (auto &s : SB) s = 127;
    run_mx("all max magnitude (+7.5)", A, B, SA, SB, wm);
    for (int i = 0; i < 32; ++i)
        for (int k = 0; k < K; ++k) A[i * K + k] = (k & 1) ? (0x20 | 0x1f) : 0x1f;  // +-7.5 alternating
    for (auto &c : B) c = 0x1f;
    for (int k = 0; k < K; k += 7)
        for (int i = 0; i < 32; ++i) A[i * K + k] = 0x01;  // 0.125 terms
    run_mx("cancellation (+-7.5 pairs, 0.125 terms)", A, B, SA, SB, wm);
    for (int i = 0; i < 32; ++i)
        for (int k = 0; k < K; ++k) A[i * K + k] = k < 32 ? 0x1f : 0x01;
    for (auto &c : B) c = 0x1f;
    for (int blk = 0; blk < K / 32; ++blk)
        for (int i = 0; i < 32; ++i) SA[blk * 32 + i] = blk == 0 ? 127 + 20 : 127 - 10;
    run_mx("one huge block + tiny blocks (scale 2^20 / 2^-10)", A, B, SA, SB, wm);
    for (auto &s : SA) s = 127;
    rnd_codes(A);
    rnd_codes(B);
    for (int blk = 0; blk < K / 32; ++blk)
        for (int i = 0; i < 32; ++i) {
            SA[blk * 32 + i] = 127 + ((blk + i) % 2 ? 12 : -12);
            SB[blk * 32 + i] = 127 + ((blk * 3 + i) % 2 ? 12 : -12);
        }
    run_mx("random codes, alternating scales 2^+-12", A, B, SA, SB, wm);

    std::printf("worst bf16 ratio %.3f (bound %.0f): %s\n", wb, 2.04 * K, wb <= 2.04 * K ? "HOLDS" : "VIOLATED");
    std::printf("worst fp6-MX ratio %.3f (allowance %.0f): %s\n", wm, 16384.0 + 3.03 * K,
                wm <= 16384.0 + 3.03 * K ? "HOLDS" : "VIOLATED");
    return (wb <= 2.04 * K && wm <= 16384.0 + 3.03 * K) ? 0 : 1;
}

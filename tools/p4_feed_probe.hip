// p4_feed_probe.hip -- how k_scan_p4m's operand feed costs the MFMA waves
// (tools only, not part of the library).
//
// One 256-thread workgroup per CU, one wave per SIMD, a 4-slot ring of 32 KiB
// LDS stages, per stage and wave 64 v_mfma_f32_16x16x32_bf16 on 8 x 8
// accumulators (the p4m tile).  Stage g's fragments are read (ds_read_b128)
// during stage g - 1; the pieces of stage g + 3 are issued during stage g; the
// stage ends with a counted vmcnt, lgkmcnt(0) and one s_barrier.
//   MODE 0  MFMA only (operands in registers, no barrier)
//   MODE 1  p4m's feed: 8 LDS-DMA pieces (4 row + 4 query) + 16 ds_read_b128
//   MODE 2  rows by LDS-DMA (4 pieces, 8 A reads), the 8 B (query) fragments
//           by global_load_dwordx4 straight into registers, issued at the
//           start of the stage before their use
//   MODE 3  no DMA: 16 ds_read_b128 + barrier (the LDS-read floor)
//   MODE 4  no DMA: 8 A reads + 8 direct B loads + barrier
//   MODE 5  MODE 3 without the barrier (16 reads + lgkmcnt(0))
//   MODE 6  barrier only (no reads, no DMA)
//   MODE 7  MODE 3 with the 16 reads early (one per 3 MFMAs over the first 48)
//   MODE 8  MODE 1 with the reads early (p4m's feed, early reads)
//   MODE 10 eight waves (two per SIMD) of 128 x 64 (feed8_body below)
//   MODE 9  MODE 3 without the lgkmcnt(0) before the barrier (the compiler
//           waits at the first use, in the next stage)
// Rows: a 4 GiB buffer streamed (4 CUs read the same tile, as p4m's query
// blocks); queries: 4 x 384 KiB blocks (L2-resident).  Random bf16 operands.
// Prints ns per stage and cycles per stage at the clock given (argv[2] GHz).
//   hipcc --offload-arch=gfx950 -O3 tools/p4_feed_probe.hip -o tools/bin/p4_feed_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int kStage = 32768, kQOff = 16384, kNbuf = 4;

__device__ inline void barrier_raw() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

template <int MODE>
__device__ __attribute__((always_inline)) inline void feed_body(const unsigned char *rows, uint64_t rmask,
                                                                const unsigned char *qs, int stages, float *out,
                                                                unsigned char *lds) {
    const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wr = w & 1, wq = w >> 1;
    const int qb = blockIdx.x & 3;
    const uint64_t grp = blockIdx.x >> 2;
    const int off = lane * 16;
    auto rsrc = [&](int g, int p) -> const void * {
        return rows + ((((grp * 1000003ull + (uint64_t)g) * 16384ull) + (uint64_t)p * 1024ull) & rmask) + off;
    };
    auto qsrc = [&](int g, int p) -> const void * {
        return qs + ((uint64_t)(qb * 24 + g % 24) * 16384ull + (uint64_t)p * 1024ull) + off;
    };
    auto issue = [&](int g, int i, bool rows_only) {
        unsigned char *dst = lds + (g % kNbuf) * kStage;
        if (i < 4) {
            __builtin_amdgcn_global_load_lds(rsrc(g, w + 4 * i), (lds_void *)(dst + (w + 4 * i) * 1024), 16, 0, 0);
        } else if (!rows_only) {
            __builtin_amdgcn_global_load_lds(qsrc(g, w + 4 * (i - 4)), (lds_void *)(dst + kQOff + (w + 4 * (i - 4)) * 1024),
                                             16, 0, 0);
        }
    };
    bf16x8 a[8], b[8], an[8], bn[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        for (int e = 0; e < 8; ++e) {
            a[i][e] = (__bf16)((float)((lane * 7 + i * 13 + e * 5) % 17) * 0.0625f - 0.5f);
            b[i][e] = (__bf16)((float)((lane * 3 + i * 11 + e * 7) % 19) * 0.0625f - 0.5f);
        }
        an[i] = a[i];
        bn[i] = b[i];
    }
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const bool dma = MODE == 1 || MODE == 2 || MODE == 8;
    // the ring holds defined bytes (else the compiler folds reads of a ring
    // that no DMA writes and re-allocates the accumulators around them)
    // (random bf16 in [-1, 1), as the streamed buffers: the clock the chip
    // holds depends on the operands)
    for (int i = t; i < kNbuf * kStage / 4; i += 256) {
        uint32_t h = (uint32_t)i * 2654435761u ^ (0x5151u + blockIdx.x);
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        const uint32_t lo = 0x3f00u | (h & 0x7fu) | ((h >> 7) & 1u) << 15;
        const uint32_t hi = 0x3f00u | ((h >> 8) & 0x7fu) | ((h >> 15) & 1u) << 15;
        reinterpret_cast<uint32_t *>(lds)[i] = lo | hi << 16;
    }
    __syncthreads();
    const bool rows_only = MODE == 2;
    // prologue: stages 0..2 issued, stage 0 landed, its fragments read
    if (dma) {
        for (int g = 0; g < 3; ++g)
            for (int i = 0; i < 8; ++i) issue(g, i, rows_only);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier_raw();
    const unsigned char *st0 = lds;
    const int rowA = wr * 8 * 1024, rowB = kQOff + wq * 8 * 1024;
    if (MODE != 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const bf16x8 *>(st0 + rowA + i * 1024 + off);
#pragma unroll
        for (int i = 0; i < 8; ++i) b[i] = *reinterpret_cast<const bf16x8 *>(st0 + rowB + i * 1024 + off);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

    auto stage = [&](int g, bf16x8(&ca)[8], bf16x8(&cb)[8], bf16x8(&na)[8], bf16x8(&nb)[8]) __attribute__((always_inline)) {
        const unsigned char *sn = lds + ((g + 1) % kNbuf) * kStage;
        if (MODE == 2 || MODE == 4) {
            // the next stage's B fragments straight from global memory
#pragma unroll
            for (int i = 0; i < 8; ++i)
                nb[i] = *reinterpret_cast<const bf16x8 *>(
                    reinterpret_cast<const unsigned char *>(qsrc(g + 1, wq * 8 + i)));
        }
#pragma unroll
        for (int x = 0; x < 64; ++x) {
            const int rb = x >> 3, jb = x & 7;
            acc[rb][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ca[rb], cb[jb], acc[rb][jb], 0, 0, 0);
            if ((MODE == 1 || MODE == 8) && (x & 7) == 4) issue(g + 3, x >> 3, false);
            if (MODE == 2 && (x & 15) == 4) issue(g + 3, x >> 4, true);
            if (MODE == 7 || MODE == 8) {
                if (x < 48 && x % 3 == 0) {
                    const int r = x / 3;  // 0..15
                    if (r < 8)
                        na[r] = *reinterpret_cast<const bf16x8 *>(sn + rowA + r * 1024 + off);
                    else
                        nb[r - 8] = *reinterpret_cast<const bf16x8 *>(sn + rowB + (r - 8) * 1024 + off);
                }
            } else if (MODE == 1 || MODE == 3 || MODE == 5 || MODE == 9) {
                if ((x & 3) == 2) {
                    const int r = x >> 2;  // 0..15
                    if (r < 8)
                        na[r] = *reinterpret_cast<const bf16x8 *>(sn + rowA + r * 1024 + off);
                    else
                        nb[r - 8] = *reinterpret_cast<const bf16x8 *>(sn + rowB + (r - 8) * 1024 + off);
                }
            } else if (MODE == 2 || MODE == 4) {
                if ((x & 7) == 2) na[x >> 3] = *reinterpret_cast<const bf16x8 *>(sn + rowA + (x >> 3) * 1024 + off);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (MODE != 0) {
            __builtin_amdgcn_sched_barrier(0);
            if (MODE == 1 || MODE == 8)
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if (MODE == 2)  // (the builtin: the compiler's waitcnt model sees it, so the
                                 // next stage's first use of the B loads needs no wait of its own)
                __builtin_amdgcn_s_waitcnt(0x0F74);  // vmcnt(4) expcnt(7) lgkmcnt(15)
            else if (MODE == 4)
                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            if (MODE != 9 && MODE != 6) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (MODE != 5) barrier_raw();
        }
        if (MODE == 0 || MODE == 6) {
            // keep the operand rotation honest without loads
#pragma unroll
            for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(na[i]), "+v"(nb[i]));
        }
    };
    for (int g = 0; g + 1 < stages; g += 2) {
        stage(g, a, b, an, bn);
        stage(g + 1, an, bn, a, b);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) s += acc[i][j][0] + acc[i][j][3];
    if (s == 1.2345f) out[t] = s;
}

#define FEED_KERNEL(M)                                                                                    \
    __global__ __launch_bounds__(256, 1) void k_feed##M(const unsigned char *rows, uint64_t rmask,             \
                                                        const unsigned char *qs, int stages, float *out) {      \
        __shared__ __attribute__((aligned(16))) unsigned char lds[kNbuf * kStage];                             \
        feed_body<M>(rows, rmask, qs, stages, out, lds);                                                       \
    }
FEED_KERNEL(0)
FEED_KERNEL(1)
FEED_KERNEL(2)
FEED_KERNEL(3)
FEED_KERNEL(4)
FEED_KERNEL(5)
FEED_KERNEL(6)
FEED_KERNEL(7)
FEED_KERNEL(8)
FEED_KERNEL(9)


// MODE 10: eight waves (two per SIMD), wave (wr, wq) = (w & 1, w >> 1) owns
// 128 rows x 64 queries (8 x 4 blocks: 128 AGPRs), 32 MFMAs per stage; the
// same 256 x 256 tile and 32 KiB stage per CU; per wave and stage 4 LDS-DMA
// pieces (2 row, 2 query) and 12 fragment reads (8 A, 4 B), read early.
// Whether the second wave on a SIMD hides the other's VMEM issue cost.
__device__ __attribute__((always_inline)) inline void feed8_body(const unsigned char *rows, uint64_t rmask,
                                                                 const unsigned char *qs, int stages, float *out,
                                                                 unsigned char *lds) {
    const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wr = w & 1, wq = w >> 1;
    const int qb = blockIdx.x & 3;
    const uint64_t grp = blockIdx.x >> 2;
    const int off = lane * 16;
    auto rsrc = [&](int g, int p) -> const void * {
        return rows + ((((grp * 1000003ull + (uint64_t)g) * 16384ull) + (uint64_t)p * 1024ull) & rmask) + off;
    };
    auto qsrc = [&](int g, int p) -> const void * {
        return qs + ((uint64_t)(qb * 24 + g % 24) * 16384ull + (uint64_t)p * 1024ull) + off;
    };
    auto issue = [&](int g, int i) {  // i 0..3: row pieces w, w + 8; query pieces w, w + 8
        unsigned char *dst = lds + (g % kNbuf) * kStage;
        const int pc = w + 8 * (i & 1);
        if (i < 2)
            __builtin_amdgcn_global_load_lds(rsrc(g, pc), (lds_void *)(dst + pc * 1024), 16, 0, 0);
        else
            __builtin_amdgcn_global_load_lds(qsrc(g, pc), (lds_void *)(dst + kQOff + pc * 1024), 16, 0, 0);
    };
    for (int i = t; i < kNbuf * kStage / 4; i += 512) {
        uint32_t h = (uint32_t)i * 2654435761u ^ (0x5151u + blockIdx.x);
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        const uint32_t lo = 0x3f00u | (h & 0x7fu) | ((h >> 7) & 1u) << 15;
        const uint32_t hi = 0x3f00u | ((h >> 8) & 0x7fu) | ((h >> 15) & 1u) << 15;
        reinterpret_cast<uint32_t *>(lds)[i] = lo | hi << 16;
    }
    __syncthreads();
    bf16x8 a[8], b[4], an[8], bn[4];
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int g = 0; g < 3; ++g)
        for (int i = 0; i < 4; ++i) issue(g, i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier_raw();
    const int rowA = wr * 8 * 1024, rowB = kQOff + wq * 4 * 1024;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const bf16x8 *>(lds + rowA + i * 1024 + off);
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = *reinterpret_cast<const bf16x8 *>(lds + rowB + i * 1024 + off);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    auto stage = [&](int g, bf16x8(&ca)[8], bf16x8(&cb)[4], bf16x8(&na)[8], bf16x8(&nb)[4]) __attribute__((always_inline)) {
        const unsigned char *sn = lds + ((g + 1) % kNbuf) * kStage;
#pragma unroll
        for (int x = 0; x < 32; ++x) {
            const int rb = x >> 2, jb = x & 3;
            acc[rb][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ca[rb], cb[jb], acc[rb][jb], 0, 0, 0);
            if ((x & 7) == 3) issue(g + 3, x >> 3);
            if (x < 24 && (x & 1) == 0) {
                const int r = x >> 1;  // 0..11
                if (r < 8)
                    na[r] = *reinterpret_cast<const bf16x8 *>(sn + rowA + r * 1024 + off);
                else
                    nb[r - 8] = *reinterpret_cast<const bf16x8 *>(sn + rowB + (r - 8) * 1024 + off);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_raw();
    };
    for (int g = 0; g + 1 < stages; g += 2) {
        stage(g, a, b, an, bn);
        stage(g + 1, an, bn, a, b);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) sum += acc[i][j][0] + acc[i][j][3];
    if (sum == 1.2345f) out[t] = sum;
}
__global__ __launch_bounds__(512, 1) void k_feed10(const unsigned char *rows, uint64_t rmask, const unsigned char *qs,
                                                   int stages, float *out) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[kNbuf * kStage];
    feed8_body(rows, rmask, qs, stages, out, lds);
}

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                               \
        }                                                                           \
    } while (0)


__global__ void k_fill(uint32_t *p, size_t n, uint32_t seed) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        // two bf16 in [-1, 1) (exponent 0x3f / 0xbf region)
        const uint32_t lo = 0x3f00u | (h & 0x7fu) | ((h >> 7) & 1u) << 15;
        const uint32_t hi = 0x3f00u | ((h >> 8) & 0x7fu) | ((h >> 15) & 1u) << 15;
        p[i] = lo | hi << 16;
    }
}

int main(int argc, char **argv) {
    const int stages = argc > 1 ? atoi(argv[1]) : 4800;
    const double ghz = argc > 2 ? atof(argv[2]) : 2.0;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t rbytes = (size_t)4 << 30, qbytes = (size_t)4 * 24 * 16384;
    unsigned char *rows = nullptr, *qs = nullptr;
    float *out = nullptr;
    CK(hipMalloc(&rows, rbytes));
    CK(hipMalloc(&qs, qbytes));
    CK(hipMalloc(&out, 4096));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)rows, rbytes / 4, 0x1234u);
    hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, (uint32_t *)qs, qbytes / 4, 0x9876u);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[] = {"mfma_only", "p4m_feed_dma8_read16", "rows_dma4_read8_direct_b8", "lds_reads16_only",
                           "read8_direct_b8_no_dma", "reads16_no_barrier", "barrier_only", "early_reads16_barrier",
                           "p4m_feed_early_reads", "reads16_barrier_no_lgkm_wait", "8waves_128x64_dma4_read12"};
    for (int mode = 0; mode < 11; ++mode) {
        auto launch = [&]() {
            if (mode == 0) hipLaunchKernelGGL(k_feed0, dim3(cus), dim3(256), 0, 0, rows, rbytes - 1, qs, stages, out);
            if (mode == 1) hipLaunchKernelGGL(k_feed1, dim3(cus), dim3(256), 0, 0, rows, rbytes - 1, qs, stages, out);
            if (mode == 2) hipLaunchKernelGGL(k_feed2, dim3(cus), dim3(256), 0, 0, rows, rbytes - 1, qs, stages, out);
            if (mode == 3) hipLaunchKernelGGL(k_feed3, dim3(cus), dim3(256), 0, 0, rows, rbytes - 1, qs, stages, out);
            if (mode == 4) hipLaunchKernelGGL(k_feed4, dim3(cus), dim3(256), 0, 0, rows, rbytes - 1, qs, stages, out);
            if (mode == 5) hipLaunchKernelGGL(k_feed5, dim3(cus), dim3(256), 0, 0, rows, rbytes - 1, qs, stages, out);
            if (mode == 6) hipLaunchKernelGGL(k_feed6, dim3(cus), dim3(256), 0, 0, rows, rbytes - 1, qs, stages, out);
            if (mode == 7) hipLaunchKernelGGL(k_feed7, dim3(cus), dim3(256), 0, 0, rows, rbytes - 1, qs, stages, out);
            if (mode == 8) hipLaunchKernelGGL(k_feed8, dim3(cus), dim3(256), 0, 0, rows, rbytes - 1, qs, stages, out);
            if (mode == 10) hipLaunchKernelGGL(k_feed10, dim3(cus), dim3(512), 0, 0, rows, rbytes - 1, qs, stages, out);
            if (mode == 9) hipLaunchKernelGGL(k_feed9, dim3(cus), dim3(256), 0, 0, rows, rbytes - 1, qs, stages, out);
        };
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f, sum = 0.f;
        const int reps = 5;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
            sum += ms;
        }
        const double ns = best * 1e6 / stages;
        const double tflops = 2.0 * 256 * 256 * 32 * (double)stages * cus / (best * 1e-3) / 1e12;
        std::printf("{\"mode\": %d, \"name\": \"%s\", \"stages\": %d, \"best_ms\": %.3f, \"mean_ms\": %.3f, "
                    "\"ns_per_stage\": %.1f, \"cycles_per_stage_at_%.2fGHz\": %.0f, \"tflops\": %.0f}\n",
                    mode, names[mode], stages, best, sum / reps, ns, ghz, ns * ghz, tflops);
        std::fflush(stdout);
    }
    return 0;
}

// l2_paths_probe.hip -- chip-wide throughput of the two ways a scan stage can
// pull L2-resident bytes into a CU (tools only, not part of the library):
//   DMA    global_load_lds_dwordx4 (1 KiB contiguous per instruction) into a
//          double-buffered LDS stage, s_waitcnt + s_barrier per stage
//   DIRECT global_load_dwordx4 into VGPRs (1 KiB contiguous per instruction),
//          folded with v_xor so the loads stay live
//   MIXED  half of the stage's bytes each way, in the same waves
// 512-thread workgroups, 1 per CU (128 KiB LDS), each wave moving STAGE_KB/8
// per stage, a working set (argv[1] KiB, default 96 MiB) swept repeatedly.
// Build: hipcc --offload-arch=gfx950 -O3 tools/l2_paths_probe.hip -o tools/l2_paths_probe.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(3))) void lds_void;
#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

constexpr int kStages = 48;
constexpr int kGroupsPerWave = 7;  // 1-KiB instructions per wave per stage (56 KiB per stage)

// MODE 0 DMA, 1 DIRECT, 2 MIXED (DMA for groups < 4, DIRECT for the rest),
// 3 DMA with group 0 of every wave streamed once from `cold` (HBM) -- 1/7 of
// the bytes miss L2, like a scan's first touch of its rows
template <int MODE>
__global__ __launch_bounds__(512) void k_paths(const uint4 *buf, int64_t nkb, unsigned *sink,
                                               const uint4 *cold = nullptr) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[2][64 * 1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t wg = blockIdx.x;
    uint4 x = make_uint4(0, 0, 0, 0);
    auto kb_of = [&](int s, int g) -> int64_t {
        return ((wg * kStages + s) * 8 * kGroupsPerWave + w * kGroupsPerWave + g) % nkb;
    };
    auto issue = [&](int s, int bf) {
#pragma unroll
        for (int g = 0; g < kGroupsPerWave; ++g) {
            const uint4 *src = buf + kb_of(s, g) * 64 + lane;
            if (MODE == 3 && g == 0) src = cold + ((wg * kStages + s) * 8 + w) * 64 + lane;
            if (MODE == 0 || MODE == 3 || (MODE == 2 && g < 4))
                __builtin_amdgcn_global_load_lds((const void *)src,
                                                 (lds_void *)&lds[bf][(w * kGroupsPerWave + g) * 1024], 16, 0, 0);
        }
    };
    // DIRECT part software-pipelined one stage ahead in registers
    uint4 nxt[kGroupsPerWave];
    auto load_regs = [&](int s) {
#pragma unroll
        for (int g = 0; g < kGroupsPerWave; ++g)
            if (MODE == 1 || (MODE == 2 && g >= 4)) nxt[g] = buf[kb_of(s, g) * 64 + lane];
    };
    issue(0, 0);
    load_regs(0);
    for (int s = 0; s < kStages; ++s) {
        if (s + 1 < kStages) issue(s + 1, (s + 1) & 1);
        if (MODE != 0) {
            uint4 cur[kGroupsPerWave];
#pragma unroll
            for (int g = 0; g < kGroupsPerWave; ++g) cur[g] = nxt[g];
            if (s + 1 < kStages) load_regs(s + 1);
#pragma unroll
            for (int g = 0; g < kGroupsPerWave; ++g) {
                if (MODE == 2 && g < 4) continue;
                x.x ^= cur[g].x;
                x.y ^= cur[g].y;
                x.z ^= cur[g].z;
                x.w ^= cur[g].w;
            }
        }
        if (MODE != 1) {
            const uint4 v = *reinterpret_cast<const uint4 *>(&lds[s & 1][w * 1024 + lane * 16]);
            x.x ^= v.x;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    }
    if ((x.x ^ x.y ^ x.z ^ x.w) == 0x12345678u) sink[threadIdx.x] = 1;
}

template <int MODE>
static void run(const char *name, const uint4 *buf, int64_t nkb, unsigned *sink, const uint4 *cold = nullptr) {
    const int grid = 256 * 64;
    hipLaunchKernelGGL(k_paths<MODE>, dim3(grid), dim3(512), 0, 0, buf, nkb, sink, cold);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_paths<MODE>, dim3(grid), dim3(512), 0, 0, buf, nkb, sink, cold);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    const double bytes = (double)grid * kStages * 8 * kGroupsPerWave * 1024.0;
    std::printf("%-12s %8.3f ms  %6.2f TB/s\n", name, best, bytes / (best * 1e-3) / 1e12);
}

int main(int argc, char **argv) {
    const int64_t nkb = argc > 1 ? std::atoll(argv[1]) : 96 * 1024;  // KiB working set
    std::printf("working set %lld KiB\n", (long long)nkb);
    uint4 *buf;
    unsigned *sink;
    CK(hipMalloc(&buf, nkb * 1024));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(buf, 1, nkb * 1024));
    run<0>("DMA", buf, nkb, sink);
    run<1>("DIRECT", buf, nkb, sink);
    run<2>("MIXED", buf, nkb, sink);
    // cold stream: grid x stages x 8 waves x 1 KiB = 6 GiB, touched once per run
    uint4 *cold;
    const size_t cold_bytes = (size_t)256 * 64 * kStages * 8 * 1024;
    CK(hipMalloc(&cold, cold_bytes));
    CK(hipMemset(cold, 2, cold_bytes));
    run<3>("DMA+1/7cold", buf, nkb, sink, cold);
    return 0;
}

// glds_mfma_probe.hip -- what an LDS-DMA piece (global_load_lds_dwordx4,
// 1 KiB per wave-instruction) costs a wave that also issues MFMAs.
//
// One 256-thread workgroup per CU (one wave per SIMD), every CU busy.  Each
// wave runs ITERS iterations of 32 v_mfma_f32_32x32x16_bf16 (16 independent
// accumulators, operands in registers) with G LDS-DMA pieces interleaved
// (one after every 32/G MFMAs) and a counted vmcnt that keeps at most 2 G
// pieces in flight.  Sources: a buffer of SRC bytes read in order (L2-resident
// at 1 MiB, HBM-streamed at 4 GiB).  Prints ns per iteration and the implied
// cycles per piece over the G = 0 loop.
//   hipcc --offload-arch=gfx950 -O3 tools/glds_mfma_probe.hip -o /tmp/glds_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;

template <int G>
__global__ __launch_bounds__(256, 1) void k_probe(const unsigned char *src, size_t src_mask, int iters,
                                                   float *out) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[65536];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    bf16x8 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a[i] = bf16x8{(__bf16)(lane * 0.001f + i), (__bf16)1.f, (__bf16)0.5f, (__bf16)0.25f,
                      (__bf16)0.125f, (__bf16)2.f, (__bf16)3.f, (__bf16)(w + 1.f)};
        b[i] = a[i];
    }
    f32x16 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{0.f};
    size_t off = ((size_t)blockIdx.x * 4 + w) * 1024 * 64 + (size_t)lane * 16;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int x = 0; x < 32; ++x) {
            acc[(x >> 2) & 3][x & 3] =
                __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[(x >> 2) & 3], b[x & 3], acc[(x >> 2) & 3][x & 3], 0, 0, 0);
            if (G > 0 && (x % (32 / (G > 0 ? G : 1))) == (32 / (G > 0 ? G : 1)) - 1) {
                const int piece = x / (32 / G);
                __builtin_amdgcn_global_load_lds((const void *)(src + (off & src_mask)),
                                                 (lds_void *)(lds + (w * 16 + piece % 16) * 1024), 16, 0, 0);
                off += 1024 * 256 * 4;  // the next piece of this wave: whole chip strides
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (G > 0) {
            if (G == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            if (G == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            if (G == 8) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            if (G == 16) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) s += acc[i][j][0];
    if (s == 1.2345f) out[threadIdx.x] = s;
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const size_t big = (size_t)4 << 30;
    unsigned char *src = nullptr;
    float *out = nullptr;
    if (hipMalloc(&src, big) != hipSuccess || hipMalloc(&out, 4096) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(src, 0, big);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct Cfg {
        const char *name;
        size_t mask;
    } cfgs[] = {{"L2-resident 1MiB", ((size_t)1 << 20) - 1}, {"HBM 4GiB", big - 1}};
    for (auto &c : cfgs) {
        double base = 0;
        for (int g : {0, 2, 4, 8, 16}) {
            auto launch = [&]() {
                switch (g) {
                    case 0: hipLaunchKernelGGL(k_probe<0>, dim3(cus), dim3(256), 0, 0, src, c.mask, iters, out); break;
                    case 2: hipLaunchKernelGGL(k_probe<2>, dim3(cus), dim3(256), 0, 0, src, c.mask, iters, out); break;
                    case 4: hipLaunchKernelGGL(k_probe<4>, dim3(cus), dim3(256), 0, 0, src, c.mask, iters, out); break;
                    case 8: hipLaunchKernelGGL(k_probe<8>, dim3(cus), dim3(256), 0, 0, src, c.mask, iters, out); break;
                    default: hipLaunchKernelGGL(k_probe<16>, dim3(cus), dim3(256), 0, 0, src, c.mask, iters, out); break;
                }
            };
            launch();
            hipDeviceSynchronize();
            float best = 1e30f;
            for (int r = 0; r < 5; ++r) {
                hipEventRecord(e0);
                launch();
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            const double ns_it = best * 1e6 / iters;
            if (g == 0) base = ns_it;
            const double gbs = g ? (double)g * 1024 * 4 * cus * iters / (best * 1e-3) / 1e9 : 0;
            printf("{\"src\": \"%s\", \"pieces_per_32_mfma\": %d, \"ns_per_iter\": %.1f, \"extra_ns_per_piece\": %.2f, "
                   "\"dma_GBps_chip\": %.0f}\n",
                   c.name, g, ns_it, g ? (ns_it - base) / g : 0.0, gbs);
        }
    }
    return 0;
}

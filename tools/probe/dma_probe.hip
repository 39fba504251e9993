// dma_probe.hip -- is the SELL-512-A value stream faster through LDS-DMA
// (global_load_lds_dwordx4 into a wave-private LDS ring) than through plain
// 16-B register loads? Values only (27 slots x 512 rows per slice, 200^3),
// one sum per row written. Not part of the product.
//
//   hipcc -O3 --offload-arch=gfx950 -o dma_probe dma_probe.hip && ./dma_probe 200 20
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);  \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

constexpr int kS = 512, kW = 27;
typedef double d2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int xcd_map(int grid)
{
    const int b = blockIdx.x, per = grid / 8;
    return (b % 8) * per + b / 8;
}

// plain register loads (the library's stream), kNT: non-temporal
template <bool kNT, int kU>
__global__ __launch_bounds__(512) void k_reg(const double* __restrict__ val, double* __restrict__ out, int nslices)
{
    const int P = xcd_map(gridDim.x);
    const int s = 2 * P + threadIdx.x / 256;
    if (s >= nslices) return;
    const int lrow = (threadIdx.x % 256) * 2;
    const double* vp = val + (size_t)s * kW * kS + lrow;
    d2v sum = {0.0, 0.0};
#pragma unroll kU
    for (int j = 0; j < kW; j++) {
        const d2v v = kNT ? __builtin_nontemporal_load((const d2v*)(vp + (size_t)j * kS)) : *(const d2v*)(vp + (size_t)j * kS);
        sum = sum + v;
    }
    *(d2v*)(out + s * kS + lrow) = sum;
}

__device__ __forceinline__ void vm_wait(int n)
{
    switch (n) {
#define W(i) case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
        W(0) W(1) W(2) W(3) W(4) W(5) W(6) W(7) W(8) W(9) W(10) W(11) W(12) W(13) W(14) W(15)
        W(16) W(17) W(18) W(19) W(20) W(21) W(22) W(23) W(24) W(25) W(26)
#undef W
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// LDS-DMA: every wave streams its own 128 rows' slots through a private ring of
// kR 1-KB entries (lane l's 16 B land at entry + 16 l: lane-linear, read back
// by the same lane with one ds_read_b128). kAux: cache policy bits (2 = nt).
template <int kR, int kAux, int kThreads>
__global__ __launch_bounds__(kThreads) void k_dma(const double* __restrict__ val, double* __restrict__ out, int nslices)
{
    __shared__ __attribute__((aligned(16))) double ring[kThreads / 64][kR][128];
    constexpr int kWavesPerSlice = 4;  // 256 rows... 4 waves x 128 rows = one slice
    const int wave = threadIdx.x / 64, lane = threadIdx.x & 63;
    constexpr int kSlicesPerBlock = kThreads / 256;
    const int B = xcd_map(gridDim.x);
    const int s = kSlicesPerBlock * B + wave / kWavesPerSlice;
    if (s >= nslices) return;
    const int lrow = (wave % kWavesPerSlice) * 128 + lane * 2;
    const double* vp = val + (size_t)s * kW * kS + lrow;
    double* r = &ring[wave][0][0];
#pragma unroll
    for (int j = 0; j < kR; j++)
        __builtin_amdgcn_global_load_lds((const void*)(vp + (size_t)j * kS), (__attribute__((address_space(3))) void*)(r + j * 128), 16, 0, kAux);
    d2v sum = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < kW; j++) {
        // entry j % kR has landed when at most issued - (j + 1) DMAs are outstanding
        vm_wait((j + kR < kW ? j + kR : kW) - j - 1);
        const d2v v = *(const d2v*)(r + (j % kR) * 128 + lane * 2);
        sum = sum + v;
        if (j + kR < kW) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_global_load_lds((const void*)(vp + (size_t)(j + kR) * kS),
                                             (__attribute__((address_space(3))) void*)(r + (j % kR) * 128), 16, 0, kAux);
        }
    }
    *(d2v*)(out + s * kS + lrow) = sum;
}

__global__ void k_gen(double* val, size_t total)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < total) val[i] = (double)(i % 7) - 3.0;
}

int main(int argc, char** argv)
{
    const int N = argc > 1 ? atoi(argv[1]) : 200;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const long long n = (long long)N * N * N;
    const int nslices = (int)((n + kS - 1) / kS);
    const size_t nval = (size_t)nslices * kW * kS;
    double *val, *out;
    CK(hipMalloc(&val, nval * 8));
    CK(hipMalloc(&out, (size_t)nslices * kS * 8));
    k_gen<<<(unsigned)((nval + 255) / 256), 256>>>(val, nval);
    CK(hipDeviceSynchronize());
    std::vector<double> ref((size_t)nslices * kS), h((size_t)nslices * kS);
    const double bytes = (double)nval * 8 + (double)nslices * kS * 8;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    bool have_ref = false;
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; i++) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; i++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1000.0 * ms / reps;
        CK(hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost));
        bool ok = true;
        if (!have_ref) {
            ref = h;
            have_ref = true;
        } else {
            for (size_t i = 0; i < h.size(); i++)
                if (h[i] != ref[i]) { ok = false; break; }
        }
        printf("%-26s %8.1f us  %7.0f GB/s %s\n", name, us, bytes / us * 1e-3, ok ? "ok" : "MISMATCH");
        fflush(stdout);
    };
    const int np = (nslices + 1) / 2, gp = (np + 7) / 8 * 8;
    run("reg nt u27", [&] { k_reg<true, 27><<<gp, 512>>>(val, out, nslices); });
    run("reg nt u6", [&] { k_reg<true, 6><<<gp, 512>>>(val, out, nslices); });
    run("reg def u27", [&] { k_reg<false, 27><<<gp, 512>>>(val, out, nslices); });
    run("dma nt R4 t512", [&] { k_dma<4, 2, 512><<<gp, 512>>>(val, out, nslices); });
    run("dma nt R8 t512", [&] { k_dma<8, 2, 512><<<gp, 512>>>(val, out, nslices); });
    run("dma nt R16 t512", [&] { k_dma<16, 2, 512><<<gp, 512>>>(val, out, nslices); });
    run("dma def R8 t512", [&] { k_dma<8, 0, 512><<<gp, 512>>>(val, out, nslices); });
    const int g1 = (nslices + 7) / 8 * 8;
    run("dma nt R4 t256", [&] { k_dma<4, 2, 256><<<g1, 256>>>(val, out, nslices); });
    run("dma nt R8 t256", [&] { k_dma<8, 2, 256><<<g1, 256>>>(val, out, nslices); });
    run("dma nt R16 t256", [&] { k_dma<16, 2, 256><<<g1, 256>>>(val, out, nslices); });
    run("reg nt u27 (again)", [&] { k_reg<true, 27><<<gp, 512>>>(val, out, nslices); });
    return 0;
}

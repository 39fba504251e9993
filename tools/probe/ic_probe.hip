// ic_probe.hip -- does the 100^3 CG iteration's value stream stay in the
// 256 MiB Infinity Cache if part of it is loaded non-temporally? Standalone
// (not part of the product): a 27-slot SELL-512-like value table (216 MB at
// 100^3), x = r + beta * p_old read at the 27 stencil offsets, p_new written
// into a rotating ring, Ap written, then an r update pass; slices below
// `split` load their values with nt loads, the rest with the default policy.
//
//   hipcc -O3 --offload-arch=gfx950 -o ic_probe ic_probe.hip
//   ./ic_probe [n=100] [iters=60]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);       \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

constexpr int kS = 512;
constexpr int kW = 27;

struct Off {
    int o[kW];
};

__global__ __launch_bounds__(kS) void k_spmv(const double* __restrict__ val, const double* __restrict__ r,
                                            const double* __restrict__ pold, double* __restrict__ p,
                                            double* __restrict__ Ap, int n, int split, int nt_vec, Off off,
                                            double beta) {
    const int s = blockIdx.x;
    const int i = s * kS + threadIdx.x;
    const double* v = val + (size_t)s * kW * kS + threadIdx.x;
    double acc = 0.0;
    const bool nt = s < split;
#pragma unroll
    for (int j = 0; j < kW; ++j) {
        int c = i + off.o[j];
        c = c < 0 ? 0 : (c >= n ? n - 1 : c);
        const double x = r[c] + beta * pold[c];
        const double a = nt ? __builtin_nontemporal_load(v + j * kS) : v[j * kS];
        acc += a * x;
    }
    if (i < n) {
        const double pn = r[i] + beta * pold[i];
        if (nt_vec) {
            __builtin_nontemporal_store(pn, p + i);
            __builtin_nontemporal_store(acc, Ap + i);
        } else {
            p[i] = pn;
            Ap[i] = acc;
        }
    }
}

__global__ __launch_bounds__(256) void k_upd(double* __restrict__ r, const double* __restrict__ Ap, int n,
                                            double alpha) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) r[i] = r[i] - alpha * Ap[i];
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 100;
    const int iters = argc > 2 ? atoi(argv[2]) : 60;
    const int n = N * N * N;
    const int nsl = (n + kS - 1) / kS;
    const int ring = 32;
    Off off;
    int j = 0;
    for (int dz = -1; dz <= 1; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) off.o[j++] = dz * N * N + dy * N + dx;
    double *val, *r, *pr, *Ap;
    CK(hipMalloc(&val, (size_t)nsl * kW * kS * 8));
    CK(hipMalloc(&r, (size_t)n * 8));
    CK(hipMalloc(&pr, (size_t)n * 8 * ring));
    CK(hipMalloc(&Ap, (size_t)n * 8));
    CK(hipMemset(val, 0x3f, (size_t)nsl * kW * kS * 8));
    CK(hipMemset(r, 0, (size_t)n * 8));
    CK(hipMemset(pr, 0, (size_t)n * 8 * ring));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)nsl * kW * kS * 8 + 4.0 * n * 8 + 3.0 * n * 8;
    const int splits[] = {0, nsl / 4, nsl / 2, 3 * nsl / 4, nsl};
    for (int nt_vec = 0; nt_vec < 2; ++nt_vec)
        for (int split : splits) {
            for (int rep = 0; rep < 2; ++rep) {
                for (int k = 0; k < 5 + iters; ++k) {
                    if (k == 5) CK(hipEventRecord(e0));
                    double* po = pr + (size_t)(k % ring) * n;
                    double* pn = pr + (size_t)((k + 1) % ring) * n;
                    k_spmv<<<nsl, kS>>>(val, r, po, pn, Ap, n, split, nt_vec, off, 0.5);
                    k_upd<<<(n + 255) / 256, 256>>>(r, Ap, n, 1e-3);
                }
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double us = 1000.0 * ms / iters;
                if (rep == 1)
                    printf("n=%d nt_vec=%d nt_slices=%d/%d  %.2f us/iter  %.0f GB/s compulsory\n", N, nt_vec, split,
                           nsl, us, bytes / us / 1e3);
            }
        }
    return 0;
}

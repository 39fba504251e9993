// capture_probe.hip -- which multi-stream hipGraph capture patterns does this
// ROCm accept? (the in-process rank group crashed inside graph capture):
//   A: one side stream forked/joined per iteration by events (the RCCL rank's
//      halo stream)
//   B: P member streams forked from stream 0, each with a side stream, events
//      re-recorded every iteration, D2D copies between members, a group-sum
//      kernel on stream 0 (the in-process group's iteration)
//   C: as B, all work on stream 0 (serialised capture)
//   hipcc -O2 --offload-arch=gfx950 -o capture_probe capture_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            printf("  HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);  \
            return 1;                                                                \
        }                                                                            \
    } while (0)

__global__ void k_add(double* a, int n, double v)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] += v;
}

__global__ void k_sum(double** loc, int P, double* out)
{
    double s = 0;
    for (int r = 0; r < P; r++) s += loc[r][0];
    *out = s;
}

int run(int mode, int P, int iters)
{
    const int n = 4096;
    std::vector<hipStream_t> s(P), s2(P);
    std::vector<hipEvent_t> ev(P + 1), ev_pb(P), ev_halo(P), ev_join(P);
    std::vector<double*> buf(P);
    for (int r = 0; r < P; r++) {
        CK(hipStreamCreateWithFlags(&s[r], hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&s2[r], hipStreamNonBlocking));
        CK(hipEventCreateWithFlags(&ev_pb[r], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&ev_halo[r], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&ev_join[r], hipEventDisableTiming));
        CK(hipMalloc(&buf[r], (n + 256) * sizeof(double)));
        CK(hipMemset(buf[r], 0, (n + 256) * sizeof(double)));
    }
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipEvent_t fork;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    double** dloc;
    CK(hipMalloc(&dloc, P * sizeof(double*)));
    CK(hipMemcpy(dloc, buf.data(), P * sizeof(double*), hipMemcpyHostToDevice));
    double* out;
    CK(hipMalloc(&out, 8));
    auto S = [&](int r) { return mode == 2 ? s[0] : s[r]; };
    auto S2 = [&](int r) { return mode == 2 ? s[0] : (mode == 0 ? s2[r] : s2[r]); };
    hipGraph_t g;
    CK(hipStreamBeginCapture(s[0], hipStreamCaptureModeThreadLocal));
    CK(hipEventRecord(fork, s[0]));
    for (int r = 1; r < P; r++) CK(hipStreamWaitEvent(S(r), fork, 0));
    for (int it = 0; it < iters; it++) {
        for (int r = 0; r < P; r++) {
            hipLaunchKernelGGL(k_add, dim3(n / 256), dim3(256), 0, S(r), buf[r], n, 1.0);
            CK(hipEventRecord(ev_pb[r], S(r)));
        }
        for (int r = 0; r < P; r++) {
            bool joined = false;
            if (r > 0) {
                CK(hipStreamWaitEvent(S2(r), ev_pb[r - 1], 0));
                CK(hipMemcpyAsync(buf[r] + n, buf[r - 1], 64 * sizeof(double), hipMemcpyDeviceToDevice, S2(r)));
                joined = true;
            }
            if (r < P - 1) {
                CK(hipStreamWaitEvent(S2(r), ev_pb[r + 1], 0));
                CK(hipMemcpyAsync(buf[r] + n + 64, buf[r + 1], 64 * sizeof(double), hipMemcpyDeviceToDevice, S2(r)));
                joined = true;
            }
            if (!joined) CK(hipStreamWaitEvent(S2(r), ev_pb[r], 0));
            CK(hipEventRecord(ev_halo[r], S2(r)));
        }
        for (int r = 0; r < P; r++) {
            hipLaunchKernelGGL(k_add, dim3(n / 256), dim3(256), 0, S(r), buf[r], n / 2, 0.5);
            CK(hipStreamWaitEvent(S(r), ev_halo[r], 0));
            hipLaunchKernelGGL(k_add, dim3(n / 256), dim3(256), 0, S(r), buf[r] + n / 2, n / 2, 0.5);
        }
        // group sum on stream 0
        for (int r = 0; r < P; r++) CK(hipEventRecord(ev[r], S(r)));
        for (int r = 1; r < P; r++) CK(hipStreamWaitEvent(S(0), ev[r], 0));
        hipLaunchKernelGGL(k_sum, dim3(1), dim3(1), 0, S(0), dloc, P, out);
        CK(hipEventRecord(ev[P], S(0)));
        for (int r = 1; r < P; r++) CK(hipStreamWaitEvent(S(r), ev[P], 0));
    }
    for (int r = 1; r < P; r++) {
        CK(hipEventRecord(ev_join[r], S(r)));
        CK(hipStreamWaitEvent(s[0], ev_join[r], 0));
    }
    CK(hipStreamEndCapture(s[0], &g));
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int k = 0; k < 3; k++) CK(hipGraphLaunch(ge, s[0]));
    CK(hipStreamSynchronize(s[0]));
    double h = 0;
    CK(hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost));
    printf("  mode %d P %d iters %d ok, sum %.1f\n", mode, P, iters, h);
    return 0;
}

int main()
{
    const int which = getenv("PROBE_MODE") ? atoi(getenv("PROBE_MODE")) : 2;
    for (int mode : {which})
        for (int P : {1, 2, 3, 8}) {
            printf("mode %d P %d ...\n", mode, P);
            fflush(stdout);
            run(mode, P, 8);
            fflush(stdout);
        }
    return 0;
}

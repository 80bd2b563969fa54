// Microbenchmark: does a hipGraph captured with a forked side stream run the side branch
// concurrently with the main chain?  Main chain: 5 dependent small launches per step; side
// branch: one 16.8 MB weight stream per step (joined back one step later).
//   hipcc --offload-arch=gfx950 -O3 -o fork fork.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

__global__ __launch_bounds__(1024) void k_small(float* out, const float* in) {
    __shared__ float red[1024];
    const float v = in[threadIdx.x + blockIdx.x * 1024];
    red[threadIdx.x] = v;
    __syncthreads();
    out[threadIdx.x + blockIdx.x * 1024] = red[1023 - threadIdx.x] + 1.f;
}

template <int CH>
__global__ __launch_bounds__(1024) void k_stream(float* out, const float* in, const float4* W) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float4* p = W + ((size_t)(blockIdx.x * 16 + wave) * CH) * 64 + lane;
    float4 w[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) w[c] = p[c * 64];
    const float x = in[threadIdx.x];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += x * (w[c].x + w[c].y + w[c].z + w[c].w);
    __shared__ float red[1024];
    red[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x < 16) {
        float t = 0.f;
        for (int k = 0; k < 64; ++k) t += red[threadIdx.x * 64 + k];
        out[blockIdx.x * 16 + threadIdx.x] = t;
    }
}

int main() {
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    float *x0, *x1, *y;
    CK(hipMalloc(&x0, 1 << 22));
    CK(hipMalloc(&x1, 1 << 22));
    CK(hipMalloc(&y, 1 << 22));
    CK(hipMemset(x0, 0, 1 << 22));
    CK(hipMemset(x1, 0, 1 << 22));
    float4* W;
    const size_t wbytes = (size_t)256 * 16 * 4 * 1024 * 4;  // 4 x 16.8 MB regions
    CK(hipMalloc(&W, wbytes));
    CK(hipMemset(W, 0, wbytes));
    hipEvent_t evf[2], evj[2];
    for (int i = 0; i < 2; ++i) {
        CK(hipEventCreateWithFlags(&evf[i], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&evj[i], hipEventDisableTiming));
    }
    const int steps = 100;
    for (int mode = 0; mode < 4; ++mode) {
        // mode 0: main chain only; 1: + side stream kernels on a forked branch; 2: side kernels
        // serialized in the main chain; 3: side only (forked)
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        float* b[2] = {x0, x1};
        for (int t = 0; t < steps; ++t) {
            if (mode != 3)
                for (int k = 0; k < 5; ++k)
                    hipLaunchKernelGGL(k_small, dim3(k == 1 || k == 3 ? 256 : 16), dim3(1024), 0, s, b[(k + 1) & 1], b[k & 1]);
            const float4* Wt = W + (size_t)(t & 3) * 256 * 16 * 4 * 64;
            if (mode == 1 || mode == 3) {
                CK(hipEventRecord(evf[t & 1], s));
                CK(hipStreamWaitEvent(s2, evf[t & 1], 0));
                hipLaunchKernelGGL(k_stream<4>, dim3(256), dim3(1024), 0, s2, y, x0, Wt);
                CK(hipEventRecord(evj[t & 1], s2));
                if (t > 0 || mode == 3) CK(hipStreamWaitEvent(s, evj[(t + 1) & 1], 0));
            } else if (mode == 2) {
                hipLaunchKernelGGL(k_stream<4>, dim3(256), dim3(1024), 0, s, y, x0, Wt);
            }
        }
        if (mode == 1 || mode == 3) CK(hipStreamWaitEvent(s, evj[(steps - 1) & 1], 0));
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
        hipEvent_t a, z;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&z));
        CK(hipEventRecord(a, s));
        for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(z, s));
        CK(hipEventSynchronize(z));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, z));
        const char* names[4] = {"main chain only (5 launches)", "main + forked side stream", "main + side serialized",
                                "side only (forked)"};
        printf("%-32s %7.2f us/step\n", names[mode], 1000.f * ms / (10 * steps));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}

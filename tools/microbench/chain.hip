// Microbenchmark: per-launch cost of a dependent chain of short kernels captured in a hipGraph
// (the decoder step's structure).  Prints us per launch for several kernel bodies.
//   hipcc --offload-arch=gfx950 -O3 -o chain chain.hip && ./chain
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

__global__ void k_empty(float*, const float*) {}

// one load of the predecessor's output + one store
__global__ void k_ldst(float* out, const float* in) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    out[i] = in[i] + 1.f;
}

// like the GEMV epilogue: load, LDS round trip with two barriers, store one value per WG
__global__ __launch_bounds__(1024) void k_lds(float* out, const float* in) {
    __shared__ float red[16][64][4];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const float v = in[i];
    red[threadIdx.x >> 6][threadIdx.x & 63][0] = v;
    __syncthreads();
    float s = 0.f;
    if (threadIdx.x < 256)
        for (int w = 0; w < 16; ++w) s += red[w][threadIdx.x & 63][threadIdx.x >> 6];
    __syncthreads();
    if (threadIdx.x < 16) out[blockIdx.x * 16 + threadIdx.x] = s;
}

// GEMV-like weight stream: each wave loads `chunks` KiB of a large read-only buffer + the input
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

template <typename F>
float time_chain(hipStream_t s, int n, F launch) {
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < n; ++i) launch(i);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int w = 0; w < 3; ++w) (void)hipGraphLaunch(ge, s);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, s);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) (void)hipGraphLaunch(ge, s);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    return 1000.f * ms / (reps * n);
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float *x0, *x1;
    const size_t nx = 256 * 1024;
    CK(hipMalloc(&x0, nx * 4));
    CK(hipMalloc(&x1, nx * 4));
    CK(hipMemset(x0, 0, nx * 4));
    CK(hipMemset(x1, 0, nx * 4));
    float4* W;
    const size_t wbytes = (size_t)256 * 16 * 10 * 1024;  // 42 MB: 256 WGs x 16 waves x 10 KiB
    CK(hipMalloc(&W, wbytes));
    CK(hipMemset(W, 0, wbytes));
    const int n = 200;
    float* buf[2] = {x0, x1};
    struct Case {
        const char* name;
        float us;
    };
    std::vector<Case> res;
    res.push_back({"empty 1 WG x 64", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, buf[i & 1], buf[(i + 1) & 1]);
                   })});
    res.push_back({"empty 256 WG x 1024", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_empty, dim3(256), dim3(1024), 0, s, buf[i & 1], buf[(i + 1) & 1]);
                   })});
    res.push_back({"ld/st 1 WG x 1024", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_ldst, dim3(1), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1]);
                   })});
    res.push_back({"ld/st 16 WG x 1024", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_ldst, dim3(16), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1]);
                   })});
    res.push_back({"ld/st 256 WG x 1024", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_ldst, dim3(256), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1]);
                   })});
    res.push_back({"ld/st 256 WG x 256", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_ldst, dim3(256), dim3(256), 0, s, buf[(i + 1) & 1], buf[i & 1]);
                   })});
    res.push_back({"lds-reduce 16 WG x 1024", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_lds, dim3(16), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1]);
                   })});
    res.push_back({"lds-reduce 256 WG x 1024", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_lds, dim3(256), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1]);
                   })});
    res.push_back({"stream 1KiB/wave 256 WG (4 MB)", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_stream<1>, dim3(256), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1], W);
                   })});
    res.push_back({"stream 4KiB/wave 256 WG (16.8 MB)", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_stream<4>, dim3(256), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1], W);
                   })});
    res.push_back({"stream 7KiB/wave 256 WG (29.4 MB)", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_stream<7>, dim3(256), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1], W);
                   })});
    res.push_back({"stream 10KiB/wave 256 WG (42 MB)", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_stream<10>, dim3(256), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1], W);
                   })});
    res.push_back({"stream 10KiB/wave 128 WG (21 MB)", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_stream<10>, dim3(128), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1], W);
                   })});
    // weight stream carved from one large allocation (page-fragment / TLB-reach check)
    float4* big;
    const size_t bigbytes = (size_t)512 << 20;
    CK(hipMalloc(&big, bigbytes));
    CK(hipMemset(big, 0, bigbytes));
    res.push_back({"big: stream 10KiB/wave 256 WG (42 MB)", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_stream<10>, dim3(256), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1], big);
                   })});
    res.push_back({"big: stream 8KiB/wave 256 WG (33.6 MB)", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_stream<8>, dim3(256), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1], big);
                   })});
    res.push_back({"big: stream 9KiB/wave 256 WG (37.7 MB)", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_stream<9>, dim3(256), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1], big);
                   })});
    // the step's pattern: 29.4 MB then 42 MB from disjoint regions, alternating (per launch)
    res.push_back({"big: alt 29.4 MB / 42 MB regions", time_chain(s, n, [&](int i) {
                       if (i & 1)
                           hipLaunchKernelGGL(k_stream<10>, dim3(256), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1],
                                              big + (64 << 20) / 16);
                       else
                           hipLaunchKernelGGL(k_stream<7>, dim3(256), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1], big);
                   })});
    // 42 MB as two 21 MB launches
    res.push_back({"big: 42 MB as 2 x 21 MB launches", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_stream<10>, dim3(128), dim3(1024), 0, s, buf[(i + 1) & 1], buf[i & 1],
                                          big + (size_t)(i & 1) * 128 * 16 * 10 * 64);
                   })});
    // 2 WGs per CU (512 WG x 512 threads, 10 KiB per wave, 42 MB)
    res.push_back({"stream 10KiB/wave 512 WG x 512 (42 MB)", time_chain(s, n, [&](int i) {
                       hipLaunchKernelGGL(k_stream<10>, dim3(512), dim3(512), 0, s, buf[(i + 1) & 1], buf[i & 1], big);
                   })});
    for (auto& r : res) printf("%-40s %7.2f us/launch\n", r.name, r.us);
    return 0;
}

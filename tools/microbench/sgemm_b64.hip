// Where does a batch-64 decoder GEMM launch spend its time?  The dec_lstm shape (K 2560, N 4096,
// B 64: 256 workgroups x 16 waves, four m-tiles per wave, two register stages of 2 chunks) with
// ingredients removed one at a time, each timed as a 200-launch dependent chain in a hipGraph.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../your-voice-tts_amd/csrc \
//         -o sgemm_b64 sgemm_b64.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "common.h"

using namespace tts;

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

constexpr int K = 2560, N = 4096, B = 64, NT = 4, NW = 16;

// V bits: 1 = load W, 2 = load X, 4 = MFMA, 8 = LDS reduction + store, 16 = X in fragment order
// (chunk c, m-tile mt: 64 lanes x float4 contiguous, one coalesced 1 KiB per load instead of 16
// rows x 64 B)
template <int V, int WAVES, int UP = 2, int ST = 2>
__global__ __launch_bounds__(WAVES * 64) void k(const float* __restrict__ W, const float* __restrict__ X, float* out) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ntile = blockIdx.x;
    const int nchunks = K / 16;
    const int cbeg = wave * nchunks / WAVES, cend = (wave + 1) * nchunks / WAVES;
    const float4* Wp = reinterpret_cast<const float4*>(W) + (size_t)ntile * nchunks * 64 + lane;
    const float* xb = X + (lane & 15) * K + (lane >> 4) * 4;
    floatx4 acc[NT];
    for (int mt = 0; mt < NT; ++mt) acc[mt] = floatx4{0.f, 0.f, 0.f, 0.f};
    float vsum = 0.f;
    float4 wA[UP], xA[UP][NT], wB[UP], xB[UP][NT], wC[UP], xC[UP][NT];
    auto ld = [&](int c0, float4(&wv)[UP], float4(&xv)[UP][NT]) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < UP; ++u) {
            const int c = min(c0 + u, cend - 1);
            wv[u] = (V & 1) ? Wp[(size_t)c * 64] : float4{1.f, 1.f, 1.f, 1.f};
#pragma unroll
            for (int mt = 0; mt < NT; ++mt)
                xv[u][mt] = (V & 2) ? ((V & 16) ? reinterpret_cast<const float4*>(X)[((size_t)c * NT + mt) * 64 + lane]
                                               : *reinterpret_cast<const float4*>(xb + (size_t)mt * 16 * K + c * 16))
                                    : float4{(float)c, 1.f, 1.f, 1.f};
        }
    };
    auto mf = [&](int c0, const float4(&wv)[UP], const float4(&xv)[UP][NT]) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < UP; ++u) {
            if (c0 + u < cend) {
                if (V & 4) {
#pragma unroll
                    for (int mt = 0; mt < NT; ++mt) acc[mt] = mfma16x16x4(xv[u][mt].x, wv[u].x, acc[mt]);
#pragma unroll
                    for (int mt = 0; mt < NT; ++mt) acc[mt] = mfma16x16x4(xv[u][mt].y, wv[u].y, acc[mt]);
#pragma unroll
                    for (int mt = 0; mt < NT; ++mt) acc[mt] = mfma16x16x4(xv[u][mt].z, wv[u].z, acc[mt]);
#pragma unroll
                    for (int mt = 0; mt < NT; ++mt) acc[mt] = mfma16x16x4(xv[u][mt].w, wv[u].w, acc[mt]);
                } else {
                    vsum += wv[u].x + wv[u].y + wv[u].z + wv[u].w;
#pragma unroll
                    for (int mt = 0; mt < NT; ++mt) vsum += xv[u][mt].x + xv[u][mt].y + xv[u][mt].z + xv[u][mt].w;
                }
            }
        }
    };
    if (ST == 2) {
        if (cbeg < cend) ld(cbeg, wA, xA);
        for (int c0 = cbeg; c0 < cend; c0 += 2 * UP) {
            ld(c0 + UP, wB, xB);
            mf(c0, wA, xA);
            if (c0 + UP >= cend) break;
            ld(c0 + 2 * UP, wA, xA);
            mf(c0 + UP, wB, xB);
        }
    } else {
        if (cbeg < cend) {
            ld(cbeg, wA, xA);
            ld(cbeg + UP, wB, xB);
        }
        for (int c0 = cbeg; c0 < cend; c0 += 3 * UP) {
            ld(c0 + 2 * UP, wC, xC);
            mf(c0, wA, xA);
            if (c0 + UP >= cend) break;
            ld(c0 + 3 * UP, wA, xA);
            mf(c0 + UP, wB, xB);
            if (c0 + 2 * UP >= cend) break;
            ld(c0 + 4 * UP, wB, xB);
            mf(c0 + 2 * UP, wC, xC);
        }
    }
    acc[0][0] += vsum;
    if (V & 8) {
        __shared__ float red[NW][NT][64][4];
#pragma unroll
        for (int mt = 0; mt < NT; ++mt)
            for (int r = 0; r < 4; ++r) red[wave][mt][lane][r] = acc[mt][r];
        __syncthreads();
        for (int e = threadIdx.x; e < NT * 256; e += blockDim.x) {
            const int mt = e >> 8, l = (e >> 2) & 63, r = e & 3;
            float s = 0.f;
            for (int w = 0; w < WAVES; ++w) s += red[w][mt][l][r];
            out[(size_t)ntile * NT * 256 + e] = s;
        }
    } else {
        out[((size_t)ntile * 1024 + threadIdx.x) * 4] = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
    }
}

// rewrites the activation buffer from every CU (what the previous step launch does in the decoder)
__global__ void producer(float* X, int n, float v) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) X[i] = v;
}

template <int V, int WAVES = NW, int UP = 2, int ST = 2>
static float run_prod(hipStream_t s, const float* W, float* X, float* out, bool gemm) {
    hipGraph_t g;
    hipGraphExec_t ge;
    const int n = 200;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < n; ++i) {
        hipLaunchKernelGGL(producer, dim3(256), dim3(256), 0, s, X, B * K, (float)i);
        if (gemm) hipLaunchKernelGGL((k<V, WAVES, UP, ST>), dim3(N / 16), dim3(WAVES * 64), 0, s, W, X, out);
    }
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int w = 0; w < 2; ++w) (void)hipGraphLaunch(ge, s);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, s);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) (void)hipGraphLaunch(ge, s);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    return 1000.f * ms / (reps * n);
}

template <int V, int WAVES = NW, int UP = 2, int ST = 2>
static float run(hipStream_t s, const float* W, const float* X, float* out) {
    hipGraph_t g;
    hipGraphExec_t ge;
    const int n = 200;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL((k<V, WAVES, UP, ST>), dim3(N / 16), dim3(WAVES * 64), 0, s, W, X, out);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int w = 0; w < 2; ++w) (void)hipGraphLaunch(ge, s);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, s);
    const int reps = 5;
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
    float *W, *X, *out;
    CK(hipMalloc(&W, (size_t)N * K * 4));
    CK(hipMalloc(&X, (size_t)B * K * 4 + 4096));
    CK(hipMalloc(&out, (size_t)N / 16 * 1024 * 4 * 4));
    CK(hipMemset(W, 0, (size_t)N * K * 4));
    CK(hipMemset(X, 0, (size_t)B * K * 4 + 4096));
    printf("dec_lstm shape K=%d N=%d B=%d, %d WGs x %d waves (us per launch, dependent chain)\n", K, N, B, N / 16, NW);
    printf("  frag, 4 waves, 2 stages of 2   %7.2f\n", run<31, 4, 2, 2>(s, W, X, out));
    const float p0 = run_prod<31, 4, 2, 2>(s, W, X, out, false);
    const float p1 = run_prod<31, 4, 2, 2>(s, W, X, out, true);
    printf("  producer alone                 %7.2f\n", p0);
    printf("  producer + frag gemm           %7.2f  (gemm after a fresh X: %.2f)\n", p1, p1 - p0);
    const float p2 = run_prod<15>(s, W, X, out, true);
    printf("  producer + rows gemm (16 w)    %7.2f  (gemm after a fresh X: %.2f)\n", p2, p2 - p0);
    return 0;
}

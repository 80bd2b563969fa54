// Microbenchmark of the decoder-step GEMV launches (the library's own sgemm kernels, compiled in)
// as dependent chains in a hipGraph: per-launch cost of each decoder shape alone (weights L2/IC
// warm) and of the five-GEMV step sequence (weights streamed from the Infinity Cache).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../your-voice-tts_amd/csrc \
//         -o sgemm_chain sgemm_chain.hip ../../your-voice-tts_amd/csrc/sgemm.hip
#include <cstdio>
#include <functional>
#include <vector>

#include "sgemm.h"

using namespace tts;

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

static float time_chain(hipStream_t s, int n, const std::function<void(int)>& launch) {
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

template <typename T>
static T* dalloc(size_t n) {
    void* p = nullptr;
    if (hipMalloc(&p, n * sizeof(T) + 64) != hipSuccess) return nullptr;
    (void)hipMemset(p, 0, n * sizeof(T) + 64);
    return static_cast<T*>(p);
}


// ---- stripped-down variants of the GEMV launch, to price each ingredient
template <int V>
__global__ __launch_bounds__(1024) void k_var(const SGemmArgs a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float4* Wp = reinterpret_cast<const float4*>(a.W) + ((size_t)blockIdx.x * 16 + wave) * 64 + lane;
    float4 w = *Wp;
    float4 x = *reinterpret_cast<const float4*>(a.seg[0].p + (lane >> 4) * 4 + (lane & 15) * 0);
    int sy = 1;
    if (V >= 1) sy = a.step[1];
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
    acc = mfma16x16x4(x.x, w.x, acc);
    acc = mfma16x16x4(x.y, w.y, acc);
    acc = mfma16x16x4(x.z, w.z, acc);
    acc = mfma16x16x4(x.w, w.w, acc);
    if (sy == 0) return;
    if (V >= 2) {
        __shared__ float red[16][64][4];
        __shared__ float fin[16][17];
        red[wave][lane][0] = acc[0]; red[wave][lane][1] = acc[1]; red[wave][lane][2] = acc[2]; red[wave][lane][3] = acc[3];
        __syncthreads();
        if (threadIdx.x < 256) {
            const int l = threadIdx.x >> 2, r = threadIdx.x & 3;
            float s = 0.f;
            for (int k = 0; k < 16; ++k) s += red[k][l][r];
            fin[(l >> 4) * 4 + r][l & 15] = s;
        }
        __syncthreads();
        if (threadIdx.x < 16) a.out[blockIdx.x * 16 + threadIdx.x] = fin[0][threadIdx.x];
    } else {
        if (lane < 16) a.out[(blockIdx.x * 16 + wave) * 16 + lane] = acc[0];
    }
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int B = 1;
    struct Shape {
        const char* name;
        int role, K, N;
    };
    const Shape shapes[] = {
        {"prenet2 K256 N256", ROLE_PRENET, 256, 256},
        {"att_lstm K1792 N4096", ROLE_ATT_LSTM, 1792, 4096},
        {"query K1024 N128", ROLE_QUERY, 1024, 128},
        {"dec_lstm K2560 N4096", ROLE_DEC_LSTM, 2560, 4096},
        {"mel(linear) K1536 N337", ROLE_MEL, 1536, 337},
    };
    int* state = dalloc<int>(4);
    int one[4] = {0, 1, 0, 1};
    CK(hipMemcpy(state, one, sizeof(one), hipMemcpyHostToDevice));
    int* done = dalloc<int>(64);
    float* x = dalloc<float>(64 * 4096);
    float* y = dalloc<float>(64 * 4096);
    float* cell = dalloc<float>(64 * 4096);
    std::vector<SGemmArgs> args;
    for (const Shape& sh : shapes) {
        SGemmArgs a{};
        a.seg[0] = Seg{x, sh.K, sh.K};
        a.nseg = 1;
        a.W = dalloc<float>(sgemm_packed_floats(sh.N, sh.K));
        a.K = sh.K;
        a.N = sh.N;
        a.B = B;
        a.bias = dalloc<float>(sh.N + 16);
        a.out = y;
        a.ldo = sh.role == ROLE_ATT_LSTM || sh.role == ROLE_DEC_LSTM ? 1024 : sh.N;
        a.out_par = -1;
        a.cell = cell;
        a.ldc = 1024;
        a.step = state;
        a.done = done;
        if (!a.W || !a.bias) return 1;
        args.push_back(a);
    }
    const int n = 240;
    for (size_t i = 0; i < args.size(); ++i) {
        const float us = time_chain(s, n, [&](int) { (void)sgemm_launch(args[i], shapes[i].role, s); });
        printf("%-28s alone      %7.2f us/launch\n", shapes[i].name, us);
    }
    const float us = time_chain(s, n, [&](int k) {
        const int i = k % 5;
        (void)sgemm_launch(args[i], shapes[i].role, s);
    });
    printf("%-28s %7.2f us/launch  (%.2f us per 5-launch step)\n", "step sequence", us, 5 * us);
    {
        SGemmArgs v = args[0];
        const float a0 = time_chain(s, n, [&](int) { hipLaunchKernelGGL(k_var<0>, dim3(16), dim3(1024), 0, s, v); });
        const float a1 = time_chain(s, n, [&](int) { hipLaunchKernelGGL(k_var<1>, dim3(16), dim3(1024), 0, s, v); });
        const float a2 = time_chain(s, n, [&](int) { hipLaunchKernelGGL(k_var<2>, dim3(16), dim3(1024), 0, s, v); });
        printf("var0 (load+mfma+store, 400B args) %7.2f us/launch\n", a0);
        printf("var1 (+ step-state load)          %7.2f us/launch\n", a1);
        printf("var2 (+ LDS 2-barrier reduction)  %7.2f us/launch\n", a2);
    }
    return 0;
}

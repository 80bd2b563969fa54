// The library's own batched decoder GEMM launch (sgemm_launch, fragment mirrors) at the B=64
// dec_lstm shape, as a 200-launch dependent chain: three input segments as in the decoder step vs
// one, zero vs random data, to compare with the stripped kernel of sgemm_b64.hip.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../your-voice-tts_amd/csrc \
//         -o sgemm_lib_b64 sgemm_lib_b64.hip ../../your-voice-tts_amd/csrc/sgemm.hip
#include <cstdio>
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

static float chain(hipStream_t s, const SGemmArgs& a, int role) {
    hipGraph_t g;
    hipGraphExec_t ge;
    const int n = 200;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < n; ++i) (void)sgemm_launch(a, role, s);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int w = 0; w < 2; ++w) (void)hipGraphLaunch(ge, s);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < 5; ++r) (void)hipGraphLaunch(ge, s);
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    return 1000.f * ms / (5 * n);
}

__global__ void fill(float* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 13;
        h *= 0x5bd1e995u;
        p[i] = ((h >> 8) & 0xffff) * (1.f / 65536.f) - 0.5f;
    }
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int B = 64, H = 1024, E = 512, K = H + E + H, N = 4 * H, NTF = 4;
    auto alloc = [](size_t n) {
        float* p = nullptr;
        (void)hipMalloc(&p, n * sizeof(float) + 256);
        (void)hipMemset(p, 0, n * sizeof(float) + 256);
        return p;
    };
    float* W = alloc(sgemm_packed_floats(N, K));
    float* bias = alloc(N);
    float* rows = alloc((size_t)B * K);
    float* mir = alloc((size_t)NTF * 16 * K);
    float* out = alloc((size_t)B * H);
    float* outf = alloc((size_t)NTF * 16 * H);
    float* cell = alloc((size_t)B * H);
    int* state = nullptr;
    CK(hipMalloc(&state, 64));
    int one[4] = {0, 1, 0, 1};
    CK(hipMemcpy(state, one, sizeof(one), hipMemcpyHostToDevice));
    int* done = nullptr;
    CK(hipMalloc(&done, 64 * sizeof(int)));
    CK(hipMemset(done, 0, 64 * sizeof(int)));
    SGemmArgs a{};
    a.B = B;
    a.K = K;
    a.N = N;
    a.W = W;
    a.bias = bias;
    a.out = out;
    a.ldo = H;
    a.out_par = -1;
    a.cell = cell;
    a.ldc = H;
    a.step = state;
    a.done = done;
    a.ntf = NTF;
    a.outf = outf;
    const size_t fc = (size_t)NTF * 256;
    a.seg[0] = Seg{rows, K, H, mir};
    a.seg[1] = Seg{rows + H, K, E, mir + (H / 16) * fc};
    a.seg[2] = Seg{rows + H + E, K, H, mir + ((H + E) / 16) * fc};
    a.nseg = 3;
    printf("library sgemm_launch, dec_lstm B=64 over mirrors (us per launch)\n");
    printf("  3 segments, zero data     %7.2f\n", chain(s, a, ROLE_DEC_LSTM));
    SGemmArgs one_seg = a;
    one_seg.seg[0] = Seg{rows, K, K, mir};
    one_seg.nseg = 1;
    printf("  1 segment, zero data      %7.2f\n", chain(s, one_seg, ROLE_DEC_LSTM));
    hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, s, W, sgemm_packed_floats(N, K), 1u);
    hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, s, mir, (size_t)NTF * 16 * K, 2u);
    hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, s, rows, (size_t)B * K, 3u);
    CK(hipStreamSynchronize(s));
    printf("  3 segments, random data   %7.2f\n", chain(s, a, ROLE_DEC_LSTM));
    printf("  1 segment, random data    %7.2f\n", chain(s, one_seg, ROLE_DEC_LSTM));
    SGemmArgs nof = a;
    nof.outf = nullptr;
    printf("  3 segments, no out mirror %7.2f\n", chain(s, nof, ROLE_DEC_LSTM));
    for (int kk : {1280, 640, 256}) {
        SGemmArgs v = one_seg;
        v.K = kk;
        v.seg[0] = Seg{rows, K, kk, mir};
        printf("  1 segment, K=%-4d          %7.2f\n", kk, chain(s, v, ROLE_DEC_LSTM));
    }
    SGemmArgs rowsonly = a;
    for (int i = 0; i < 3; ++i) rowsonly.seg[i].pf = nullptr;
    printf("  row-major (16 waves)      %7.2f\n", chain(s, rowsonly, ROLE_DEC_LSTM));
    return 0;
}

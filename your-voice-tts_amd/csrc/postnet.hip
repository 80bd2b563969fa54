// Postnet (layers/tacotron2.py:30-45) + residual (models/tacotron2.py:69-70) as five
// LDS-tiled fp32 MFMA implicit GEMMs (conv1d k=5, "same" padding per sentence length).
//
//   out[b][t][co] = epi( sum_{k<5} sum_{ci} in[b][t+k-2][ci] * W[co][ci][k] ),  in = 0 outside [0, T_b)
//   epi: BatchNorm (eval) folded to acc*scale + shift, tanh on layers 0-3, + mel on layer 4.
// Activations are time-major [B][T][C] (channels contiguous), the layout the decoder writes.
// Roofline: MFMA-fp32 bound, 8.68 MFLOP per frame.
#include <vector>

#include "common.h"

using namespace tts;

namespace {

constexpr int BM = 64;  // frames per tile
constexpr int BN = 64;  // output channels per tile
constexpr int BK = 16;  // input channels per K step
constexpr int KW = 5;   // kernel width
constexpr int PAD = 2;

// Packed weights: [ci][k][co_pad] (co contiguous); co_pad = Cout rounded up to BN.
__global__ void pack_conv_kernel(const float* W, int Cout, int Cin, int co_pad, float* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)Cin * KW * co_pad;
    if (i >= total) return;
    const int co = i % co_pad;
    const int k = (i / co_pad) % KW;
    const int ci = i / ((int64_t)co_pad * KW);
    out[i] = co < Cout ? W[((int64_t)co * Cin + ci) * KW + k] : 0.f;
}

// scale = gamma / sqrt(var + eps); shift = beta + (bias - mean) * scale
__global__ void fold_bn_kernel(const float* bias, const float* gamma, const float* beta, const float* mean,
                               const float* var, int C, float* scale, float* shift) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float sc = gamma[c] / sqrtf(var[c] + 1e-5f);
    scale[c] = sc;
    shift[c] = beta[c] + (bias[c] - mean[c]) * sc;
}

struct ConvArgs {
    const float* in;  // [B][Tmax][Cin]
    float* out;       // [B][Tmax][Cout]
    const float* W;   // packed [Cin][5][co_pad]
    const float* scale;
    const float* shift;
    const float* resid;  // [B][Tmax][Cout] or null
    const int* T;        // [B]
    int Tmax, Cin, Cout, co_pad, act_tanh;
};

__global__ __launch_bounds__(256) void conv_k5_kernel(const ConvArgs a) {
    const int b = blockIdx.z;
    const int t0 = blockIdx.x * BM;
    const int c0 = blockIdx.y * BN;
    const int Tb = a.T[b];
    if (t0 >= Tb) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wt = (wave >> 1) * 32;  // wave's frame offset in tile
    const int wc = (wave & 1) * 32;   // wave's channel offset in tile
    __shared__ float xs[BM + 2 * PAD][BK + 1];
    __shared__ float ws[BK][KW][BN];
    // one accumulator set per kernel tap: five 512-long fma chains instead of one 2560-long
    // chain keeps the fp32 accumulation error near the reference's blocked CPU convolution
    floatx4 acc[KW][2][2];
#pragma unroll
    for (int k = 0; k < KW; ++k)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[k][i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const float* inb = a.in + (int64_t)b * a.Tmax * a.Cin;
    for (int ci0 = 0; ci0 < a.Cin; ci0 += BK) {
        // stage input rows t0-2 .. t0+BM+1, channels ci0 .. ci0+15 (zero outside [0, T_b))
        for (int i = tid; i < (BM + 2 * PAD) * (BK / 4); i += blockDim.x) {
            const int r = i / (BK / 4), c4 = i % (BK / 4);
            const int t = t0 - PAD + r;
            float4 v = float4{0.f, 0.f, 0.f, 0.f};
            if (t >= 0 && t < Tb) v = *reinterpret_cast<const float4*>(inb + (int64_t)t * a.Cin + ci0 + c4 * 4);
            xs[r][c4 * 4 + 0] = v.x;
            xs[r][c4 * 4 + 1] = v.y;
            xs[r][c4 * 4 + 2] = v.z;
            xs[r][c4 * 4 + 3] = v.w;
        }
        // stage weights [ci0..ci0+15][k][c0..c0+63]
        for (int i = tid; i < BK * KW * (BN / 4); i += blockDim.x) {
            const int c4 = i % (BN / 4);
            const int rk = i / (BN / 4);  // ci_local*5 + k
            const float4 v = *reinterpret_cast<const float4*>(a.W + ((int64_t)(ci0 * KW + rk)) * a.co_pad + c0 + c4 * 4);
            *reinterpret_cast<float4*>(&ws[rk / KW][rk % KW][c4 * 4]) = v;
        }
        __syncthreads();
        const int row = lane & 15, kq = lane >> 4;
#pragma unroll
        for (int k = 0; k < KW; ++k) {
#pragma unroll
            for (int kk = 0; kk < BK; kk += 4) {
                float av[2], bv[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) av[i] = xs[wt + i * 16 + row + k][kk + kq];
#pragma unroll
                for (int j = 0; j < 2; ++j) bv[j] = ws[kk + kq][k][wc + j * 16 + row];
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[k][i][j] = mfma16x16x4(av[i], bv[j], acc[k][i][j]);
            }
        }
        __syncthreads();
    }
    // epilogue: D lane l holds C[(l>>4)*4 + r][l&15]  (row = frame, col = channel)
    float* outb = a.out + (int64_t)b * a.Tmax * a.Cout;
    const float* resb = a.resid ? a.resid + (int64_t)b * a.Tmax * a.Cout : nullptr;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int t = t0 + wt + i * 16 + (lane >> 4) * 4 + r;
                const int co = c0 + wc + j * 16 + (lane & 15);
                if (t < Tb && co < a.Cout) {
                    float sum = acc[0][i][j][r];
#pragma unroll
                    for (int k = 1; k < KW; ++k) sum += acc[k][i][j][r];
                    float y = sum * a.scale[co] + a.shift[co];
                    if (a.act_tanh) y = tanhf(y);
                    if (resb) y = resb[(int64_t)t * a.Cout + co] + y;
                    outb[(int64_t)t * a.Cout + co] = y;
                }
            }
}

}  // namespace

struct tts_postnet {
    int n_mel = 80;
    int cin[5], cout[5], co_pad[5];
    float* W[5] = {};
    float* scale[5] = {};
    float* shift[5] = {};
    float* buf[2] = {};
    size_t buf_floats = 0;
    int* T = nullptr;
    int Tcap_B = 0;
};

extern "C" {

void tts_postnet_destroy(tts_postnet* p) {
    if (!p) return;
    for (int i = 0; i < 5; ++i) {
        if (p->W[i]) (void)hipFree(p->W[i]);
        if (p->scale[i]) (void)hipFree(p->scale[i]);
        if (p->shift[i]) (void)hipFree(p->shift[i]);
    }
    for (int i = 0; i < 2; ++i)
        if (p->buf[i]) (void)hipFree(p->buf[i]);
    if (p->T) (void)hipFree(p->T);
    delete p;
}

tts_status tts_postnet_create(const tts_tensor* tensors, int n_tensors, int n_mel, void* stream, tts_postnet** out) {
    TTS_CHECK(tensors && out && n_mel > 0 && n_mel % 16 == 0, TTS_ERR_INVALID, "bad postnet arguments");
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto* p = new tts_postnet();
    p->n_mel = n_mel;
    const int ch[6] = {n_mel, 512, 512, 512, 512, n_mel};
    auto find = [&](const std::string& key, int64_t numel) -> const float* {
        for (int i = 0; i < n_tensors; ++i)
            if (key == tensors[i].key) {
                if (tensors[i].numel != numel) { set_error("weight " + key + " has wrong size"); return nullptr; }
                return tensors[i].data;
            }
        set_error("missing weight " + key);
        return nullptr;
    };
    for (int l = 0; l < 5; ++l) {
        const std::string pre = "postnet.convolutions." + std::to_string(l) + ".net.";
        const int ci = ch[l], co = ch[l + 1];
        p->cin[l] = ci;
        p->cout[l] = co;
        p->co_pad[l] = (co + BN - 1) / BN * BN;
        const float* w = find(pre + "0.weight", (int64_t)co * ci * KW);
        const float* bias = find(pre + "0.bias", co);
        const float* g = find(pre + "1.weight", co);
        const float* be = find(pre + "1.bias", co);
        const float* mu = find(pre + "1.running_mean", co);
        const float* var = find(pre + "1.running_var", co);
        if (!w || !bias || !g || !be || !mu || !var) { tts_postnet_destroy(p); return TTS_ERR_INVALID; }
        const int64_t nw = (int64_t)ci * KW * p->co_pad[l];
        if (hipMalloc(&p->W[l], nw * 4) != hipSuccess || hipMalloc(&p->scale[l], co * 4) != hipSuccess ||
            hipMalloc(&p->shift[l], co * 4) != hipSuccess) {
            tts_postnet_destroy(p);
            set_error("hipMalloc failed");
            return TTS_ERR_NOMEM;
        }
        hipLaunchKernelGGL(pack_conv_kernel, dim3((nw + 255) / 256), dim3(256), 0, s, w, co, ci, p->co_pad[l], p->W[l]);
        hipLaunchKernelGGL(fold_bn_kernel, dim3((co + 255) / 256), dim3(256), 0, s, bias, g, be, mu, var, co,
                           p->scale[l], p->shift[l]);
    }
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) { tts_postnet_destroy(p); return hip_fail(e, "postnet pack", __FILE__, __LINE__); }
    *out = p;
    return TTS_OK;
}

tts_status tts_postnet_run(tts_postnet* p, const float* mel, const int32_t* T, int B, int Tmax, float* out,
                           void* stream) {
    TTS_CHECK(p && mel && T && out && B >= 1 && Tmax >= 1, TTS_ERR_INVALID, "bad postnet_run arguments");
    for (int b = 0; b < B; ++b) TTS_CHECK(T[b] >= 0 && T[b] <= Tmax, TTS_ERR_INVALID, "T[b] out of range");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t need = (size_t)B * Tmax * 512;
    if (need > p->buf_floats) {
        for (int i = 0; i < 2; ++i) {
            if (p->buf[i]) (void)hipFree(p->buf[i]);
            p->buf[i] = nullptr;
            TTS_HIP(hipMalloc(&p->buf[i], need * 4));
        }
        p->buf_floats = need;
    }
    if (B > p->Tcap_B) {
        if (p->T) (void)hipFree(p->T);
        p->T = nullptr;
        TTS_HIP(hipMalloc(&p->T, B * sizeof(int)));
        p->Tcap_B = B;
    }
    TTS_HIP(hipMemcpyAsync(p->T, T, B * sizeof(int), hipMemcpyHostToDevice, s));
    const float* in = mel;
    for (int l = 0; l < 5; ++l) {
        ConvArgs a{};
        a.in = in;
        a.out = l == 4 ? out : p->buf[l & 1];
        a.W = p->W[l];
        a.scale = p->scale[l];
        a.shift = p->shift[l];
        a.resid = l == 4 ? mel : nullptr;
        a.T = p->T;
        a.Tmax = Tmax;
        a.Cin = p->cin[l];
        a.Cout = p->cout[l];
        a.co_pad = p->co_pad[l];
        a.act_tanh = l < 4;
        hipLaunchKernelGGL(conv_k5_kernel, dim3((Tmax + BM - 1) / BM, p->co_pad[l] / BN, B), dim3(256), 0, s, a);
        TTS_HIP(hipGetLastError());
        in = a.out;
    }
    return TTS_OK;
}

}  // extern "C"

// Skinny fp32 MFMA GEMM + fused LSTM cell epilogue (see sgemm.h for the layout).
//
// Replaces, per decoder step (layers/tacotron2.py:194-224, common_layers.py:77-83,170):
//   attention_rnn / decoder_rnn  nn.LSTMCell  (gates GEMV + pointwise, fused here)
//   prenet linear+relu, query_layer, linear_projection.
// Roofline at B <= ~40: HBM/Infinity-Cache bound on the weight stream (each packed weight
// byte is read exactly once per step by exactly one wave).
#include "sgemm.h"

namespace tts {

constexpr int MAX_WAVES = 8;

// ROLE only names the instantiation (distinct kernel names in rocprof traces per decoder stage).
template <int MT, int EPI, int ROLE>
__global__ __launch_bounds__(512) void sgemm_kernel(const SGemmArgs a) {
    if (a.n_active && *a.n_active == 0) return;
    const int ntile = blockIdx.x;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int nw = blockDim.x >> 6;
    const int step = a.step ? *a.step : 0;
    const int nchunks = a.K >> 4;
    const int cbeg = wave * nchunks / nw;
    const int cend = (wave + 1) * nchunks / nw;

    // Per-lane activation base pointers: row b = mt*16 + (lane&15), k offset (lane>>4)*4.
    const int xrow = lane & 15;
    const int xk = (lane >> 4) * 4;
    const float* xb[3][MT];
    int cb[3];
    int kstart = 0;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
        const Seg& g = a.seg[s];
        const bool live = s < a.nseg;
        const float* p = live ? g.p + (g.par >= 0 ? (int64_t)((step + g.par) & 1) * g.pstride : 0) : nullptr;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int b = mt * 16 + xrow;
            xb[s][mt] = (live && b < a.B) ? p + (int64_t)b * g.ld + xk - kstart : nullptr;
        }
        kstart += live ? g.len : 0;
        cb[s] = kstart >> 4;  // first chunk past segment s
    }

    floatx4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = floatx4{0.f, 0.f, 0.f, 0.f};

    const float4* __restrict__ Wp = reinterpret_cast<const float4*>(a.W) + (size_t)ntile * nchunks * 64 + lane;
    constexpr int U = 4;
    for (int c0 = cbeg; c0 < cend; c0 += U) {
        float4 wv[U];
        float4 xv[U][MT];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = c0 + u;
            if (c < cend) {
                wv[u] = Wp[(size_t)c * 64];  // default policy: the 72.7 MB weight set stays in the Infinity Cache across steps
                const int s = c < cb[0] ? 0 : (c < cb[1] ? 1 : 2);
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    const float* p = s == 0 ? xb[0][mt] : (s == 1 ? xb[1][mt] : xb[2][mt]);
                    xv[u][mt] = p ? *reinterpret_cast<const float4*>(p + c * 16) : float4{0.f, 0.f, 0.f, 0.f};
                }
            } else {
                wv[u] = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) xv[u][mt] = float4{0.f, 0.f, 0.f, 0.f};
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                acc[mt] = mfma16x16x4(xv[u][mt].x, wv[u].x, acc[mt]);
                acc[mt] = mfma16x16x4(xv[u][mt].y, wv[u].y, acc[mt]);
                acc[mt] = mfma16x16x4(xv[u][mt].z, wv[u].z, acc[mt]);
                acc[mt] = mfma16x16x4(xv[u][mt].w, wv[u].w, acc[mt]);
            }
        }
    }

    // Cross-wave K reduction in a fixed order.
    __shared__ float red[MAX_WAVES][MT][64][4];
    __shared__ float fin[MT * 16][17];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        red[wave][mt][lane][0] = acc[mt].x;
        red[wave][mt][lane][1] = acc[mt].y;
        red[wave][mt][lane][2] = acc[mt].z;
        red[wave][mt][lane][3] = acc[mt].w;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < MT * 256; e += blockDim.x) {
        const int mt = e >> 8, l = (e >> 2) & 63, r = e & 3;
        float s = 0.f;
        for (int w = 0; w < nw; ++w) s += red[w][mt][l][r];
        fin[mt * 16 + (l >> 4) * 4 + r][l & 15] = s;
    }
    __syncthreads();

    const bool track = a.hist != nullptr && step < a.hist_cap;
    if (EPI == EPI_LINEAR) {
        float* out = a.out ? a.out + (a.out_par >= 0 ? (int64_t)((step + a.out_par) & 1) * a.out_pstride : 0) : nullptr;
        for (int e = threadIdx.x; e < a.B * 16; e += blockDim.x) {
            const int b = e >> 4, col = e & 15;
            const int n = ntile * 16 + col;
            if (n >= a.N) continue;
            float v = fin[b][col];
            if (a.bias) v += a.bias[n];
            if (a.act == ACT_RELU) v = fmaxf(v, 0.f);
            if (out) out[(int64_t)b * a.ldo + n] = v;
            if (a.out2) a.out2[(int64_t)b * a.ldo2 + n] = v;
            if (track && !(a.done && a.done[b])) a.hist[(int64_t)b * a.ldh + (int64_t)step * a.N + n] = v;
        }
    } else {
        // LSTM cell (torch LSTMCell, gate order i, f, g, o): c' = s(f)c + s(i)tanh(g); h' = s(o)tanh(c')
        float* out = a.out + (a.out_par >= 0 ? (int64_t)((step + a.out_par) & 1) * a.out_pstride : 0);
        for (int e = threadIdx.x; e < a.B * 4; e += blockDim.x) {
            const int b = e >> 2, u = e & 3;
            const int unit = ntile * 4 + u;
            const float* bl = a.bias + ntile * 16;
            const float gi = fin[b][u] + bl[u];
            const float gf = fin[b][4 + u] + bl[4 + u];
            const float gg = fin[b][8 + u] + bl[8 + u];
            const float go = fin[b][12 + u] + bl[12 + u];
            float* cp = a.cell + (int64_t)b * a.ldc + unit;
            const float c2 = sigmoidf_(gf) * (*cp) + sigmoidf_(gi) * tanhf(gg);
            *cp = c2;
            out[(int64_t)b * a.ldo + unit] = sigmoidf_(go) * tanhf(c2);
        }
    }
}

__global__ void sgemm_pack_kernel(const float* A, int K1, const float* Bm, int K2, int N, int rowmap, int H,
                                  float* packed, size_t total) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int K = K1 + K2;
    const int nchunks = K >> 4;
    const int j = i & 3;
    const int lane = (i >> 2) & 63;
    const size_t tc = i >> 8;  // ntile*nchunks + c
    const int c = tc % nchunks;
    const int ntile = tc / nchunks;
    const int nl = ntile * 16 + (lane & 15);
    const int k = c * 16 + (lane >> 4) * 4 + j;
    int row = nl;
    if (rowmap == ROWMAP_LSTM) {
        const int col = nl & 15, gate = col >> 2, u = col & 3;
        row = gate * H + (nl >> 4) * 4 + u;
    }
    float v = 0.f;
    if (nl < N) v = k < K1 ? A[(size_t)row * K1 + k] : Bm[(size_t)row * K2 + (k - K1)];
    packed[i] = v;
}

__global__ void sgemm_bias_kernel(const float* a, const float* b, int N, int Npad, int rowmap, int H, float* out) {
    const int nl = blockIdx.x * blockDim.x + threadIdx.x;
    if (nl >= Npad) return;
    int row = nl;
    if (rowmap == ROWMAP_LSTM) {
        const int col = nl & 15, gate = col >> 2, u = col & 3;
        row = gate * H + (nl >> 4) * 4 + u;
    }
    float v = 0.f;
    if (nl < N) v = a[row] + (b ? b[row] : 0.f);
    out[nl] = v;
}

hipError_t sgemm_pack(const float* A, int K1, const float* Bm, int K2, int N, int rowmap, int H, float* packed,
                      hipStream_t s) {
    const size_t total = sgemm_packed_floats(N, K1 + K2);
    hipLaunchKernelGGL(sgemm_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, s, A, K1, Bm, K2, N, rowmap, H,
                       packed, total);
    return hipGetLastError();
}

hipError_t sgemm_pack_bias(const float* a, const float* b, int N, int rowmap, int H, float* out, hipStream_t s) {
    const int Npad = (N + 15) / 16 * 16;
    hipLaunchKernelGGL(sgemm_bias_kernel, dim3((Npad + 255) / 256), dim3(256), 0, s, a, b, N, Npad, rowmap, H, out);
    return hipGetLastError();
}

template <int EPI, int ROLE>
static hipError_t launch_role(const SGemmArgs& a, hipStream_t s) {
    const int nchunks = a.K / 16;
    const int nw = nchunks < MAX_WAVES ? nchunks : MAX_WAVES;
    const dim3 grid((a.N + 15) / 16), block(nw * 64);
    const int mt = (a.B + 15) / 16;
    if (mt <= 1)
        hipLaunchKernelGGL((sgemm_kernel<1, EPI, ROLE>), grid, block, 0, s, a);
    else if (mt <= 2)
        hipLaunchKernelGGL((sgemm_kernel<2, EPI, ROLE>), grid, block, 0, s, a);
    else
        hipLaunchKernelGGL((sgemm_kernel<4, EPI, ROLE>), grid, block, 0, s, a);
    return hipGetLastError();
}

hipError_t sgemm_launch(const SGemmArgs& a, int role, hipStream_t s) {
    switch (role) {
        case ROLE_PRENET: return launch_role<EPI_LINEAR, ROLE_PRENET>(a, s);
        case ROLE_ATT_LSTM: return launch_role<EPI_LSTM, ROLE_ATT_LSTM>(a, s);
        case ROLE_QUERY: return launch_role<EPI_LINEAR, ROLE_QUERY>(a, s);
        case ROLE_DEC_LSTM: return launch_role<EPI_LSTM, ROLE_DEC_LSTM>(a, s);
        case ROLE_MEL: return launch_role<EPI_LINEAR, ROLE_MEL>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace tts

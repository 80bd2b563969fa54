// Non-GEMM kernels of the Tacotron / TacotronGST path (see tacotron.h):
//   bigru_kernel           GRU recurrences of the CBHG stacks (layers/tacotron.py:165-170, 204-205) and of
//                          the GST reference encoder (layers/gst_layers.py:53-56, 74-75);
//   gst_conv2d_kernel      ReferenceEncoder conv stack (gst_layers.py:35-65);
//   style_attention_kernel StyleTokenLayer + MultiHeadAttention (gst_layers.py:88-168);
//   tacotron_init_kernel   decoder / attention state init (layers/tacotron.py:336-357).
#include "tacotron.h"

namespace tts {

// ---------------------------------------------------------------- GRU recurrence
// torch GRU, ATen cell: r = s(xi_r + hh_r), z = s(xi_z + hh_z), n = tanh(xi_n + r * hh_n),
// h' = (h - n) * z + n with xi = W_ih x + b_ih (one GEMM over every position beforehand) and
// hh = W_hh h + b_hh.  One workgroup per (sentence, direction) runs the whole sequence: 768
// threads, thread (row = tid/2, half = tid%2) keeps W_hh[row][64*half, +64) in VGPRs, h lives in
// LDS (ping-pong), so a step costs two barriers and no global traffic besides xi and the output.
constexpr int GRU_THREADS = 6 * GRU_H;

__global__ __launch_bounds__(GRU_THREADS) void bigru_kernel(const GruSeqArgs a) {
    const int b = blockIdx.x, dir = blockIdx.y;
    const int tid = threadIdx.x;
    const int row = tid >> 1, half = tid & 1;
    const int Tb = a.T[b];
    __shared__ __align__(16) float hs[2][GRU_H];
    __shared__ float gs[3 * GRU_H];
    float4 w[16];
    const float4* wp = reinterpret_cast<const float4*>(a.Whh + ((int64_t)dir * 3 * GRU_H + row) * GRU_H + half * 64);
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = wp[i];
    const float bh = a.bhh[dir * 3 * GRU_H + row];
    const int xld = a.ndir * 3 * GRU_H;
    const float* xib = a.xi + (int64_t)b * a.Tmax * xld + dir * 3 * GRU_H;
    float ad1 = 0.f, ad2 = 0.f, xr = 0.f, xz = 0.f, xn = 0.f;
    if (tid < GRU_H) {
        hs[0][tid] = 0.f;
        if (a.add1) ad1 = a.add1[(int64_t)b * a.add_ld + dir * GRU_H + tid];
        if (a.add2) ad2 = a.add2[(int64_t)b * a.add_ld + dir * GRU_H + tid];
        if (Tb > 0) {
            const float* x = xib + (int64_t)(dir ? Tb - 1 : 0) * xld;
            xr = x[tid];
            xz = x[GRU_H + tid];
            xn = x[2 * GRU_H + tid];
        }
    }
    __syncthreads();
    for (int s = 0; s < Tb; ++s) {
        const int cur = s & 1;
        const float4* h4 = reinterpret_cast<const float4*>(&hs[cur][half * 64]);
        typedef float f2v __attribute__((ext_vector_type(2)));
        f2v p0 = f2v{0.f, 0.f}, p1 = p0, p2 = p0, p3 = p0;
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
            const float4 h0 = h4[i], h1 = h4[i + 1];
            p0 = __builtin_elementwise_fma(f2v{w[i].x, w[i].y}, f2v{h0.x, h0.y}, p0);
            p1 = __builtin_elementwise_fma(f2v{w[i].z, w[i].w}, f2v{h0.z, h0.w}, p1);
            p2 = __builtin_elementwise_fma(f2v{w[i + 1].x, w[i + 1].y}, f2v{h1.x, h1.y}, p2);
            p3 = __builtin_elementwise_fma(f2v{w[i + 1].z, w[i + 1].w}, f2v{h1.z, h1.w}, p3);
        }
        const float c0 = p0.x + p0.y, c1 = p1.x + p1.y, c2 = p2.x + p2.y, c3 = p3.x + p3.y;
        float g = (c0 + c1) + (c2 + c3);
        g += dpp_move<0xB1, 0xf>(g, 0.f);  // quad_perm [1,0,3,2]: the row's other half
        if (half == 0) gs[row] = g + bh;
        __syncthreads();
        if (tid < GRU_H) {
            const int pos = dir ? Tb - 1 - s : s;
            const float r = sigmoid_cell(xr + gs[tid]);
            const float z = sigmoid_cell(xz + gs[GRU_H + tid]);
            const float n = tanh_cell(xn + r * gs[2 * GRU_H + tid]);
            const float h = (hs[cur][tid] - n) * z + n;
            hs[cur ^ 1][tid] = h;
            if (a.out) a.out[((int64_t)b * a.Tmax + pos) * a.out_ld + dir * GRU_H + tid] = (h + ad1) + ad2;
            if (s + 1 < Tb) {  // next position's input projection, in flight across the barrier
                const float* x = xib + (int64_t)(dir ? Tb - 2 - s : s + 1) * xld;
                xr = x[tid];
                xz = x[GRU_H + tid];
                xn = x[2 * GRU_H + tid];
            }
        }
        __syncthreads();
    }
    if (a.h_last && tid < GRU_H) a.h_last[((int64_t)b * a.ndir + dir) * GRU_H + tid] = hs[Tb & 1][tid];
}

hipError_t launch_bigru(const GruSeqArgs& a, int B, hipStream_t s) {
    if (a.ndir < 1 || a.ndir > 2) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bigru_kernel, dim3(B, a.ndir), dim3(GRU_THREADS), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------- decoder state init
__global__ void tacotron_init_kernel(const TInitArgs a) {
    const int b = blockIdx.x;
    const int L = a.lens[b];
    for (int k = threadIdx.x; k < T_DEC; k += blockDim.x) {
        const int64_t o = a.h_pstride + (int64_t)b * T_DEC + k;
        a.h_att[o] = a.att_init[k];            // attention_rnn_init (:346-347)
        a.h1[o] = a.dec_init[k];               // decoder_rnn_inits rows 0, 1 (:348-351)
        a.h2[o] = a.dec_init[T_DEC + k];
        a.xa[(int64_t)b * T_XA + T_PRE2 + k] = 0.f;  // current_context_vec = 0 (:352)
    }
    for (int k = threadIdx.x; k < a.nmel; k += blockDim.x) a.mem[(int64_t)b * a.nmel + k] = a.mem_init[k];  // :343
    for (int j = threadIdx.x; j < a.Lcap; j += blockDim.x) {  // init_forward_attn: [1, 1e-7, ...]
        const int64_t o = (int64_t)b * a.Lcap + j;
        a.alpha[o] = j == 0 ? 1.f : (j < L ? 1e-7f : 0.f);
        a.att_w[o] = 0.f;
        a.att_cum[o] = 0.f;
    }
    if (threadIdx.x == 0) {
        a.u[b] = 0.5f;
        a.win_idx[b] = -1;
        a.nidx[b] = 1;
        a.tail[b] = 0.f;
        a.flag1[b] = 0;
        a.count[b] = 0;
        a.done[b] = 0;
        a.n_steps[b] = 0;
        if (b == 0) {
            a.state[0] = 0;
            a.state[1] = a.B;
        }
    }
}

hipError_t launch_tacotron_init(const TInitArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(tacotron_init_kernel, dim3(a.B), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------- GST reference encoder
__global__ __launch_bounds__(256) void gst_conv2d_kernel(const float* in, int Cin, int H, int W, const float* Wt,
                                                         const float* scale, const float* shift, int Cout, int Ho,
                                                         int Wo, float* out, int seq_layout) {
    const int b = blockIdx.y;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= Cout * Ho * Wo) return;
    const int co = idx / (Ho * Wo), rem = idx % (Ho * Wo), i = rem / Wo, j = rem % Wo;
    const float* inb = in + (int64_t)b * Cin * H * W;
    float s = 0.f;
    for (int ci = 0; ci < Cin; ++ci) {
        const float* wc = Wt + ((int64_t)co * Cin + ci) * 9;
        const float* ic = inb + (int64_t)ci * H * W;
#pragma unroll
        for (int ki = 0; ki < 3; ++ki) {
            const int hh = 2 * i + ki - 1;
            if (hh < 0 || hh >= H) continue;
#pragma unroll
            for (int kj = 0; kj < 3; ++kj) {
                const int ww = 2 * j + kj - 1;
                if (ww < 0 || ww >= W) continue;
                s = fmaf(wc[ki * 3 + kj], ic[hh * W + ww], s);
            }
        }
    }
    const float y = fmaxf(s * scale[co] + shift[co], 0.f);
    if (seq_layout)
        out[(((int64_t)b * Ho + i) * Cout + co) * Wo + j] = y;
    else
        out[(((int64_t)b * Cout + co) * Ho + i) * Wo + j] = y;
}

hipError_t launch_gst_conv2d(const float* in, int Cin, int H, int W, const float* Wt, const float* scale,
                             const float* shift, int Cout, float* out, int seq_layout, int B, hipStream_t s) {
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    const int n = Cout * Ho * Wo;
    hipLaunchKernelGGL(gst_conv2d_kernel, dim3((n + 255) / 256, B), dim3(256), 0, s, in, Cin, H, W, Wt, scale, shift,
                       Cout, Ho, Wo, out, seq_layout);
    return hipGetLastError();
}

// one workgroup per sentence, thread d = output unit (num_units 256, 4 heads of 64, 10 tokens)
__global__ __launch_bounds__(256) void style_attention_kernel(const float* h, const float* tokens, const float* Wq,
                                                              const float* Wk, const float* Wv, float* out) {
    const int b = blockIdx.x, d = threadIdx.x;
    __shared__ float tok[10][64];
    __shared__ float hsh[128];
    __shared__ float qs[256];
    __shared__ float ks[10][256];
    __shared__ float vs[10][256];
    __shared__ float sc[4][10];
    for (int i = d; i < 640; i += 256) tok[i / 64][i % 64] = tanhf(tokens[i]);  // tanh(style_tokens)
    if (d < 128) hsh[d] = h[(int64_t)b * 128 + d];
    __syncthreads();
    float q = 0.f;
    for (int k = 0; k < 128; ++k) q = fmaf(Wq[d * 128 + k], hsh[k], q);  // W_query (:134-142)
    qs[d] = q;
    for (int i = 0; i < 10; ++i) {  // W_key / W_value of the tokens
        float kk = 0.f, vv = 0.f;
        for (int e = 0; e < 64; ++e) {
            kk = fmaf(Wk[d * 64 + e], tok[i][e], kk);
            vv = fmaf(Wv[d * 64 + e], tok[i][e], vv);
        }
        ks[i][d] = kk;
        vs[i][d] = vv;
    }
    __syncthreads();
    if (d < 40) {  // scores = q k^T / key_dim ** 0.5 per head (:158-159)
        const int hd = d / 10, i = d % 10;
        float s = 0.f;
        for (int e = 0; e < 64; ++e) s = fmaf(qs[hd * 64 + e], ks[i][hd * 64 + e], s);
        sc[hd][i] = s / 8.0f;
    }
    __syncthreads();
    if (d < 4) {  // softmax over the 10 tokens (:160)
        float m = sc[d][0];
        for (int i = 1; i < 10; ++i) m = fmaxf(m, sc[d][i]);
        float sum = 0.f;
        for (int i = 0; i < 10; ++i) {
            const float e = expf(sc[d][i] - m);
            sc[d][i] = e;
            sum += e;
        }
        for (int i = 0; i < 10; ++i) sc[d][i] = sc[d][i] / sum;
    }
    __syncthreads();
    const int hd = d / 64;
    float o = 0.f;
    for (int i = 0; i < 10; ++i) o = fmaf(sc[hd][i], vs[i][d], o);  // scores . V, heads concatenated (:163-166)
    out[(int64_t)b * 256 + d] = o;
}

hipError_t launch_style_attention(const float* h, const float* tokens, const float* Wq, const float* Wk,
                                  const float* Wv, float* out, int B, hipStream_t s) {
    hipLaunchKernelGGL(style_attention_kernel, dim3(B), dim3(256), 0, s, h, tokens, Wq, Wk, Wv, out);
    return hipGetLastError();
}

__global__ void gather_rows_kernel(const float* table, const int* ids, int width, float* out) {
    const int b = blockIdx.x;
    const float* src = table + (int64_t)ids[b] * width;
    for (int k = threadIdx.x; k < width; k += blockDim.x) out[(int64_t)b * width + k] = src[k];
}

hipError_t launch_gather_rows(const float* table, const int* ids, int width, float* out, int B, hipStream_t s) {
    hipLaunchKernelGGL(gather_rows_kernel, dim3(B), dim3(256), 0, s, table, ids, width, out);
    return hipGetLastError();
}

__global__ void fold_pre1_stop_kernel(const float* W1, const float* b1, const float* ws, const float* bs, int nmel,
                                      float* Wf, float* bf) {
    const int K = nmel + T_DEC;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)(T_PRE1 + 1) * (K + 1)) return;
    const int n = i / (K + 1), k = i % (K + 1);
    float v;
    if (n < T_PRE1)
        v = k < K ? (k < nmel ? W1[(int64_t)n * nmel + k] : 0.f) : b1[n];
    else
        v = k < K ? (k < nmel ? ws[T_DEC + k] : ws[k - nmel]) : bs[0];
    if (k < K)
        Wf[(int64_t)n * K + k] = v;
    else
        bf[n] = v;
}

hipError_t fold_pre1_stop(const float* W1, const float* b1, const float* ws, const float* bs, int nmel, float* Wf,
                          float* bf, hipStream_t s) {
    const int64_t total = (int64_t)(T_PRE1 + 1) * (nmel + T_DEC + 1);
    hipLaunchKernelGGL(fold_pre1_stop_kernel, dim3((total + 255) / 256), dim3(256), 0, s, W1, b1, ws, bs, nmel, Wf, bf);
    return hipGetLastError();
}

__global__ void fill_int_kernel(int* p, int n, int v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

hipError_t launch_fill_int(int* p, int n, int v, hipStream_t s) {
    hipLaunchKernelGGL(fill_int_kernel, dim3((n + 255) / 256), dim3(256), 0, s, p, n, v);
    return hipGetLastError();
}

}  // namespace tts

// Decoder-step kernels other than the GEMMs: state init, processed-inputs projection,
// the attention step (one workgroup per sentence) and the stop rule.
//
// Reference: Attention.forward and helpers (layers/common_layers.py:139-256),
// Decoder._init_states / inference stop rule (layers/tacotron2.py:157-177, 256-277).
#include "decoder.h"

namespace tts {

// ------------------------------------------------------------------ init (per call)
__global__ void decoder_init_kernel(const InitArgs a) {
    const int b = blockIdx.x;
    const int L = a.lens[b];
    // step 0 reads the "previous" ping-pong slot (parity 1) for h_att / h_dec and xa[0] for ctx.
    float* ha = a.h_att + a.h_pstride + (int64_t)b * HATT;
    float* hd = a.h_dec + a.h_pstride + (int64_t)b * HDEC;
    for (int k = threadIdx.x; k < HATT; k += blockDim.x) {
        ha[k] = a.att_init[k];  // attention_rnn_init (tacotron2.py:162-163)
        a.c_att[(int64_t)b * HATT + k] = 0.f;
        hd[k] = a.dec_init[k];  // decoder_rnn_inits (tacotron2.py:167-168)
        a.c_dec[(int64_t)b * HDEC + k] = 0.f;
    }
    for (int k = threadIdx.x; k < ENC; k += blockDim.x) a.xa[(int64_t)b * XA + PRE + k] = 0.f;  // context = 0
    for (int k = threadIdx.x; k < a.nmel; k += blockDim.x) a.mem[(int64_t)b * a.nmel + k] = a.go[k];  // go frame
    // Attention.init_states / init_forward_attn (common_layers.py:139-161): alpha = [1, 1e-7, ...]
    for (int j = threadIdx.x; j < a.Lcap; j += blockDim.x) {
        const int64_t o = (int64_t)b * a.Lcap + j;
        a.alpha[o] = j == 0 ? 1.f : (j < L ? 1e-7f : 0.f);
        a.att_w[o] = 0.f;
        a.att_cum[o] = 0.f;
    }
    if (threadIdx.x == 0) {
        a.u[b] = 0.5f;
        a.win_idx[b] = -1;
        a.tail[b] = 0.f;
        a.flag1[b] = 0;
        a.count[b] = 0;
        a.done[b] = 0;
        a.n_steps[b] = 0;
        if (b == 0) {
            *a.step = 0;
            *a.n_active = a.B;
        }
    }
}

hipError_t launch_decoder_init(const InitArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(decoder_init_kernel, dim3(a.B), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------ processed inputs
// Pt[b][d][j] = sum_k W[d][k] enc[b][j][k]  (inputs_layer, common_layers.py:115-116, tacotron2.py:176)
// Stored d-major so the per-step energy loop reads it coalesced along j.
__global__ __launch_bounds__(256) void project_inputs_kernel(const float* enc, const float* W, int Lmax, int Lcap,
                                                             float* Pt) {
    const int b = blockIdx.y;
    const int j0 = blockIdx.x * 16;
    __shared__ __align__(16) float xs[16][ENC];
    for (int i = threadIdx.x; i < 16 * ENC / 4; i += blockDim.x) {
        const int r = i / (ENC / 4), c = i % (ENC / 4);
        const int j = j0 + r;
        float4 v = float4{0.f, 0.f, 0.f, 0.f};
        if (j < Lmax) v = reinterpret_cast<const float4*>(enc + ((int64_t)b * Lcap + j) * ENC)[c];
        reinterpret_cast<float4*>(&xs[r][0])[c] = v;
    }
    __syncthreads();
    const int d = threadIdx.x & 127;
    const int jh = threadIdx.x >> 7;
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    const float4* w4 = reinterpret_cast<const float4*>(W + (int64_t)d * ENC);
    for (int k4 = 0; k4 < ENC / 4; ++k4) {
        const float4 w = w4[k4];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float4 x = reinterpret_cast<const float4*>(&xs[jh * 8 + i][0])[k4];
            acc[i] += w.x * x.x + w.y * x.y + w.z * x.z + w.w * x.w;
        }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int j = j0 + jh * 8 + i;
        if (j < Lmax) Pt[((int64_t)b * ADIM + d) * Lcap + j] = acc[i];
    }
}

hipError_t launch_project_inputs(const float* enc, const float* W, int B, int Lmax, int Lcap, float* Pt,
                                 hipStream_t s) {
    hipLaunchKernelGGL(project_inputs_kernel, dim3((Lmax + 15) / 16, B), dim3(256), 0, s, enc, W, Lmax, Lcap, Pt);
    return hipGetLastError();
}

// ------------------------------------------------------------------ attention step
size_t attention_smem_bytes(int Lcap, int location) {
    size_t f = ADIM + 4 * (size_t)Lcap + 8 * (size_t)Lcap + 64;
    if (location) f += 2 * ((size_t)Lcap + 32) + (size_t)NLOC * Lcap + ADIM * NLOC;
    return f * sizeof(float);
}

// Per-thread strided partials then a block reduction (fixed order => deterministic).
__device__ __forceinline__ float strided_sum(const float* x, int n, float* scr) {
    float s = 0.f;
    for (int j = threadIdx.x; j < n; j += blockDim.x) s += x[j];
    return block_sum(s, scr);
}
__device__ __forceinline__ float strided_max(const float* x, int n, float* scr) {
    float m = -INFINITY;
    for (int j = threadIdx.x; j < n; j += blockDim.x) m = fmaxf(m, x[j]);
    return block_max(m, scr);
}
// argmax with first-index ties; `prev_shift` reads x[j-1] (0 at j=0) instead of x[j].
__device__ __forceinline__ int strided_argmax(const float* x, int n, bool prev_shift, float* scr, int* iscr) {
    float m = -INFINITY;
    int mi = 0x7fffffff;
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
        const float v = prev_shift ? (j ? x[j - 1] : 0.f) : x[j];
        if (v > m || mi == 0x7fffffff) { m = v; mi = j; }
    }
    return block_argmax(m, mi, scr, iscr);
}

__global__ __launch_bounds__(ATT_THREADS) void attention_kernel(const AttnArgs a) {
    if (*a.n_active == 0) return;
    const int b = blockIdx.x;
    const int t = *a.step;
    const int L = a.lens[b];
    const int Lc = a.Lcap;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    extern __shared__ __align__(16) float sm[];
    float* q = sm;
    float* e = q + ADIM;
    float* al = e + Lc;
    float* an = al + Lc;
    float* aold = an + Lc;
    float* red = aold + Lc;
    float* scr = red + 8 * Lc;
    int* iscr = reinterpret_cast<int*>(scr + 32);
    float* cat = scr + 64;
    float* locf = cat + 2 * (Lc + 32);
    float* wd = locf + NLOC * Lc;

    const int64_t row = (int64_t)b * Lc;
    const float* h = a.h_att + (int64_t)(t & 1) * a.h_pstride + (int64_t)b * HATT;
    for (int d = tid; d < ADIM; d += blockDim.x) q[d] = a.q[(int64_t)b * ADIM + d];
    if (a.forward_attn)
        for (int j = tid; j < L; j += blockDim.x) aold[j] = a.alpha[row + j];
    if (a.location_attn) {
        // attention_cat = [attention_weights; attention_weights_cum] (common_layers.py:167-169),
        // zero padded by (31-1)/2 = 15 on both sides for location_conv (:90-96).
        for (int j = tid; j < L + 2 * 15; j += blockDim.x) {
            const int p = j - 15;
            const bool in = p >= 0 && p < L;
            cat[j] = in ? a.att_w[row + p] : 0.f;
            cat[Lc + 32 + j] = in ? a.att_cum[row + p] : 0.f;
        }
        for (int i = tid; i < ADIM * NLOC; i += blockDim.x) wd[i] = a.loc_dense[i];
    }
    __syncthreads();
    if (a.location_attn) {
        for (int idx = tid; idx < NLOC * L; idx += blockDim.x) {
            const int f = idx / L, j = idx - f * L;
            const float* cw = a.loc_conv + f * 2 * KLOC;
            float s = 0.f;
            for (int k = 0; k < KLOC; ++k) s += cw[k] * cat[j + k];
            for (int k = 0; k < KLOC; ++k) s += cw[KLOC + k] * cat[Lc + 32 + j + k];
            locf[f * Lc + j] = s;
        }
        __syncthreads();
    }

    // energies e_j = v . tanh(pq + [loc_j] + P_j) + b_v  (common_layers.py:166-182)
    const float* Pt = a.Pt + (int64_t)b * ADIM * Lc;
    for (int j0 = 0; j0 < L; j0 += 64) {
        const int j = j0 + lane;
        if (j < L) {
            float s = 0.f;
            for (int dd = 0; dd < ADIM / 8; ++dd) {
                const int d = wave * (ADIM / 8) + dd;
                float x = q[d];
                if (a.location_attn) {
                    float lc = 0.f;
                    for (int f = 0; f < NLOC; ++f) lc += wd[d * NLOC + f] * locf[f * Lc + j];
                    x += lc;
                }
                x += Pt[(int64_t)d * Lc + j];
                s += a.v[d] * tanhf(x);
            }
            red[wave * Lc + j] = s;
        }
    }
    __syncthreads();
    const float vb = a.v_b[0];
    for (int j = tid; j < L; j += blockDim.x) {
        float s = 0.f;
        for (int w = 0; w < 8; ++w) s += red[w * Lc + j];
        e[j] = s + vb;
    }
    __syncthreads();

    // eval-mode windowing (common_layers.py:184-197)
    if (a.windowing) {
        const int wi = a.win_idx[b];
        const int back = wi - 2, front = wi + 6;
        for (int j = tid; j < L; j += blockDim.x)
            if ((back > 0 && j < back) || (front < L && j >= front)) e[j] = -INFINITY;
        __syncthreads();
        if (wi == -1) {
            const float m = strided_max(e, L, scr);
            __syncthreads();
            if (tid == 0) e[0] = m;
            __syncthreads();
        }
        const int idx = strided_argmax(e, L, false, scr, iscr);
        if (tid == 0) a.win_idx[b] = idx;
        __syncthreads();
    }

    // normalisation (common_layers.py:239-245)
    if (a.attn_norm == 0) {
        const float m = strided_max(e, L, scr);
        for (int j = tid; j < L; j += blockDim.x) al[j] = expf(e[j] - m);
        __syncthreads();
        const float s = strided_sum(al, L, scr);
        for (int j = tid; j < L; j += blockDim.x) al[j] = al[j] / s;
    } else {
        for (int j = tid; j < L; j += blockDim.x) al[j] = sigmoidf_(e[j]);
        __syncthreads();
        const float s = strided_sum(al, L, scr);
        for (int j = tid; j < L; j += blockDim.x) al[j] = al[j] / s;
    }
    __syncthreads();
    if (a.location_attn)  // update_location_attention (:163-164)
        for (int j = tid; j < L; j += blockDim.x) a.att_cum[row + j] += al[j];

    const float* w = al;
    if (a.forward_attn) {
        // apply_forward_attention (common_layers.py:199-223)
        const float u = a.u[b];
        const float omu = 1.f - u;
        for (int j = tid; j < L; j += blockDim.x) {
            const float prev = j ? aold[j - 1] : 0.f;
            const float mix = __fadd_rn(__fadd_rn(__fmul_rn(omu, aold[j]), __fmul_rn(u, prev)), 1e-8f);
            an[j] = __fmul_rn(mix, al[j]);
        }
        __syncthreads();
        if (a.forward_attn_mask) {
            const int n = strided_argmax(aold, L, true, scr, iscr);  // argmax of prev_alpha
            __syncthreads();
            const float val = strided_max(an, L, scr);
            __syncthreads();
            // Python slicing of :211-213 incl. the negative-index wrap for n < 2
            for (int j = tid; j < L; j += blockDim.x) {
                const bool z = (j >= n + 3) || (n >= 1 ? j < n - 1 : j < L - 1);
                if (z) an[j] = 0.f;
            }
            __syncthreads();
            if (tid == 0) an[(n - 2 + L) % L] = 0.01f * val;
            __syncthreads();
        }
        const float s = strided_sum(an, L, scr);
        for (int j = tid; j < L; j += blockDim.x) an[j] = an[j] / s;
        __syncthreads();
        w = an;
        for (int j = tid; j < L; j += blockDim.x) a.alpha[row + j] = an[j];
    }

    // context = w . inputs  (bmm, common_layers.py:217 / 253)
    float* ctx_out = a.xa + (int64_t)((t + 1) & 1) * a.xa_pstride + (int64_t)b * XA + PRE;
    const float* encb = a.enc + row * ENC;
    float ctx = 0.f;
    {
        const int d = tid;  // blockDim == 512 == ENC
        int j = 0;
        for (; j + 4 <= L; j += 4) {
            const float e0 = encb[(int64_t)(j + 0) * ENC + d];
            const float e1 = encb[(int64_t)(j + 1) * ENC + d];
            const float e2 = encb[(int64_t)(j + 2) * ENC + d];
            const float e3 = encb[(int64_t)(j + 3) * ENC + d];
            ctx += w[j] * e0;
            ctx += w[j + 1] * e1;
            ctx += w[j + 2] * e2;
            ctx += w[j + 3] * e3;
        }
        for (; j < L; ++j) ctx += w[j] * encb[(int64_t)j * ENC + d];
        ctx_out[d] = ctx;
    }
    if (a.forward_attn && a.trans_agent) {
        // u = sigmoid(ta([context, query]))  (:220-222)
        float p = a.ta_w[tid] * ctx;
        for (int k = tid; k < HATT; k += blockDim.x) p += a.ta_w[ENC + k] * h[k];
        const float s = block_sum(p, scr);
        if (tid == 0) a.u[b] = sigmoidf_(s + a.ta_b[0]);
    }
    // attention_weights: alpha (forward) or alignment; history; stop-rule tail (tacotron2.py:268)
    const bool rec = !a.done[b] && t < a.hist_cap && a.align_hist;
    for (int j = tid; j < a.Lalign; j += blockDim.x) {
        const float v = j < L ? w[j] : 0.f;
        if (j < L && a.location_attn) a.att_w[row + j] = v;
        if (rec) a.align_hist[(int64_t)b * a.align_ldb + (int64_t)t * a.Lalign + j] = v;
    }
    if (tid == 0) a.tail[b] = L >= 2 ? w[L - 2] + w[L - 1] : w[0];
}

hipError_t launch_attention(const AttnArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(attention_kernel, dim3(a.B), dim3(ATT_THREADS), attention_smem_bytes(a.Lcap, a.location_attn),
                       s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------ stopnet + stop rule
// stop = sigmoid(stopnet([h_dec; mel]))   (tacotron2.py:219-224, 262)
// flags as tacotron2.py:257-277: stop_flags[0] is always true; [1] latches
// (tail > 0.8 and t > L); [2] = t > 2L; 20 extra steps; cap checked only in the `elif`.
__global__ __launch_bounds__(256) void stop_kernel(const StopArgs a) {
    if (*a.n_active == 0) return;
    const int t = *a.step;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int b = wave; b < a.B; b += nw) {
        if (a.done[b]) continue;
        const float* h = a.h_dec + (int64_t)(t & 1) * a.h_pstride + (int64_t)b * HDEC;
        const float* m = a.mem + (int64_t)b * a.nmel;
        float p = 0.f;
        for (int k = lane; k < HDEC; k += 64) p += a.w[k] * h[k];
        for (int k = lane; k < a.nmel; k += 64) p += a.w[HDEC + k] * m[k];
        p = wave_sum(p);
        if (lane == 0) {
            const float st = sigmoidf_(p + a.b[0]);
            if (t < a.hist_cap) a.stop_hist[(int64_t)b * a.stop_ldb + t] = st;
            const int L = a.lens[b];
            const int f1 = a.flag1[b] | ((a.tail[b] > 0.8f && t > L) ? 1 : 0);
            a.flag1[b] = f1;
            const bool f2 = t > 2 * L;
            if (f1 && f2) {
                const int c = a.count[b] + 1;
                a.count[b] = c;
                if (c > 20) { a.done[b] = 1; a.n_steps[b] = t + 1; }
            } else if (t + 1 == a.max_steps) {
                a.done[b] = 1;
                a.n_steps[b] = t + 1;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int n = 0;
        for (int b = 0; b < a.B; ++b) n += a.done[b] ? 0 : 1;
        *a.n_active = n;
        *a.step = t + 1;
    }
}

hipError_t launch_stop(const StopArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(stop_kernel, dim3(1), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace tts

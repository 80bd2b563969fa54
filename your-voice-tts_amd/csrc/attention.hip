// Decoder-step kernels other than the GEMMs: state init, processed-inputs projection and the
// attention step (one workgroup per sentence).
//
// Reference: Attention.forward and helpers (layers/common_layers.py:139-256),
// Decoder._init_states (layers/tacotron2.py:157-177).
#include "decoder.h"

namespace tts {

// ------------------------------------------------------------------ init (per call)
// workgroup `bid` of the init (bid < B: sentence bid's state; else the resident hand-off granules)
__device__ __forceinline__ void decoder_init_block(const InitArgs& a, int bid) {
    if (bid >= a.B) {  // the extra workgroups zero the resident hand-off granules
        for (int i = (bid - a.B) * blockDim.x + threadIdx.x; i < a.nzero; i += INIT_ZERO_BLOCKS * blockDim.x)
            a.zero[i] = 0ull;
        return;
    }
    const int b = bid;
    const int L = a.lens[b];
    if (a.pre1_go && !a.keep)
        for (int k = threadIdx.x; k < PRE; k += blockDim.x) a.pre1[(int64_t)b * PRE + k] = a.pre1_go[k];
    // step 0 reads the "previous" ping-pong slot (parity 1) for h_att / h_dec and xa[0] for ctx.
    float* ha = a.h_att + a.h_pstride + (int64_t)b * HATT;
    float* hd = a.h_dec + a.h_pstride + (int64_t)b * HDEC;
    for (int k = threadIdx.x; k < HATT && !a.keep; k += blockDim.x) {
        ha[k] = a.att_init[k];  // attention_rnn_init (tacotron2.py:162-163)
        a.c_att[(int64_t)b * HATT + k] = 0.f;
        hd[k] = a.dec_init[k];  // decoder_rnn_inits (tacotron2.py:167-168)
        a.c_dec[(int64_t)b * HDEC + k] = 0.f;
    }
    if (!a.keep) {
        for (int k = threadIdx.x; k < ENC; k += blockDim.x) a.xa[(int64_t)b * XA + PRE + k] = 0.f;  // context = 0
        for (int k = threadIdx.x; k < a.nmel; k += blockDim.x) a.mem[(int64_t)b * a.nmel + k] = a.go[k];  // go frame
    }
    // Attention.init_states / init_forward_attn (common_layers.py:139-161): alpha = [1, 1e-7, ...]
    for (int j = threadIdx.x; j < a.Lcap; j += blockDim.x) {
        const int64_t o = (int64_t)b * a.Lcap + j;
        a.alpha[o] = j == 0 ? 1.f : (j < L ? 1e-7f : 0.f);
        a.att_w[o] = 0.f;
        a.att_cum[o] = 0.f;
    }
    if (a.locf)  // location_conv of zero attention state
        for (int k = threadIdx.x; k < NLOC * a.Lcap; k += blockDim.x) a.locf[(int64_t)b * NLOC * a.Lcap + k] = 0.f;
    if (threadIdx.x == 0) {
        a.u[b] = 0.5f;
        a.win_idx[b] = -1;
        a.nidx[b] = 1;  // argmax of prev_alpha = [0, 1, 1e-7, ...]
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
__global__ void decoder_init_kernel(const InitArgs a) { decoder_init_block(a, blockIdx.x); }

hipError_t launch_decoder_init(const InitArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(decoder_init_kernel, dim3(a.B + (a.zero ? INIT_ZERO_BLOCKS : 0)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// Teacher forcing (Decoder.forward, layers/tacotron2.py:227-247): the memory of step t is the go
// frame at t = 0 (left by decoder_init_kernel) and teacher row t-1 otherwise (_reshape_memory:
// frames (t-1) r .. t r - 1 of sentence b, contiguous in [B][T][80]); t comes from the device step slot.
__global__ void teacher_memory_kernel(const float* frames, int64_t ldb, int width, const int* step, float* mem) {
    const int b = blockIdx.x;
    const int t = step[0];
    if (t == 0) return;
    const float* src = frames + (int64_t)b * ldb + (int64_t)(t - 1) * width;
    for (int k = threadIdx.x; k < width; k += blockDim.x) mem[(int64_t)b * width + k] = src[k];
}

hipError_t launch_teacher_memory(const float* frames, int64_t ldb, int width, const int* step, float* mem, int B,
                                 hipStream_t s) {
    hipLaunchKernelGGL(teacher_memory_kernel, dim3(B), dim3(128), 0, s, frames, ldb, width, step, mem);
    return hipGetLastError();
}

// Zero rows [n_steps[b], nmax) of a per-sentence history dst[b][step][width].
__global__ void zero_tail_kernel(float* dst, int64_t ldb, const int* n_steps, int width, int nmax) {
    const int b = blockIdx.x;
    float* p = dst + (int64_t)b * ldb;
    for (int64_t i = (int64_t)n_steps[b] * width + threadIdx.x; i < (int64_t)nmax * width; i += blockDim.x) p[i] = 0.f;
}

hipError_t launch_zero_tail(float* dst, int64_t ldb, const int* n_steps, int width, int nmax, int B, hipStream_t s) {
    hipLaunchKernelGGL(zero_tail_kernel, dim3(B), dim3(256), 0, s, dst, ldb, n_steps, width, nmax);
    return hipGetLastError();
}

// ------------------------------------------------------------------ processed inputs
// Pt[b][d][j] = sum_k W[d][k] enc[b][j][k]  (inputs_layer, common_layers.py:115-116, tacotron2.py:176)
// Stored d-major so the per-step energy loop reads it coalesced along j.
// Workgroup = 32 attention dims x PJ_POS positions; each dim's 512-long dot products are split over
// 8 adjacent lanes (K slices of ENC_ / 8, every W load of a lane issued at once) and reduced with
// xor shuffles in a fixed order: a short dependency chain per thread instead of one W row streamed
// serially.  Grid (ADIM / 32 dim groups x position tiles, B).
constexpr int PJ_POS = 8;
constexpr int PJ_KS = 8;   // K slices per dim
constexpr int PJ_DG = 32;  // dims per workgroup
template <int ENC_>
__global__ __launch_bounds__(256) void project_inputs_kernel(const float* enc, const float* W, int Lmax, int Lcap,
                                                             float* Pt) {
    constexpr int KQ = ENC_ / 4 / PJ_KS;  // float4 per lane
    const int b = blockIdx.y;
    const int dg = blockIdx.x % (ADIM / PJ_DG);
    const int j0 = (blockIdx.x / (ADIM / PJ_DG)) * PJ_POS;
    const int tid = threadIdx.x, ks = tid & (PJ_KS - 1), d = dg * PJ_DG + (tid >> 3);
    __shared__ __align__(16) float xs[PJ_POS][ENC_];
    const float4* w4 = reinterpret_cast<const float4*>(W + (int64_t)d * ENC_) + ks * KQ;
    float4 w[KQ];
#pragma unroll
    for (int q = 0; q < KQ; ++q) w[q] = w4[q];
    constexpr int XL = PJ_POS * ENC_ / 4 / 256;
#pragma unroll
    for (int t = 0; t < XL; ++t) {
        const int i = tid + t * 256;
        const int r = i / (ENC_ / 4), c = i % (ENC_ / 4);
        const int j = j0 + r;
        float4 v = float4{0.f, 0.f, 0.f, 0.f};
        if (j < Lmax) v = reinterpret_cast<const float4*>(enc + ((int64_t)b * Lcap + j) * ENC_)[c];
        reinterpret_cast<float4*>(&xs[r][0])[c] = v;
    }
    __syncthreads();
    float acc[PJ_POS];
#pragma unroll
    for (int i = 0; i < PJ_POS; ++i) {
        acc[i] = 0.f;
#pragma unroll
        for (int q = 0; q < KQ; ++q) {
            const float4 x = reinterpret_cast<const float4*>(&xs[i][0])[ks * KQ + q];
            acc[i] += w[q].x * x.x + w[q].y * x.y + w[q].z * x.z + w[q].w * x.w;
        }
    }
#pragma unroll
    for (int o = 1; o < PJ_KS; o <<= 1)
#pragma unroll
        for (int i = 0; i < PJ_POS; ++i) acc[i] += __shfl_xor(acc[i], o, 64);
    // every lane of the 8 holds the same sums (the xor butterfly adds commutative pairs); lane ks
    // stores position ks
    float v = acc[0];
#pragma unroll
    for (int i = 1; i < PJ_POS; ++i) v = ks == i ? acc[i] : v;
    if (j0 + ks < Lmax) Pt[((int64_t)b * ADIM + d) * Lcap + j0 + ks] = v;
}
static_assert(PJ_POS == PJ_KS, "one stored position per K-slice lane");

// The same projection on the matrix cores (round 5; the VALU form above ran 12 us at L = 100 on
// 52 workgroups): P^T[j][d] = enc[j] . W[d] as 16 x 16 output tiles (16 positions x 16 dims) of
// v_mfma_f32_16x16x4_f32 (exact fp32 products), one workgroup per tile, K split over its four
// waves and the partial tiles summed in wave order.  K is walked in groups of four k-steps so a
// lane's operands are float4 loads: k-step (u, v) has lane (row, q) at k = K0 + 16 u + 4 q + v,
// the same k for A (an encoder row) and B (a W row) -- a permutation of the sum, not of its terms.
template <int ENC_>
__device__ __forceinline__ void project_tile(const float* enc, const float* W, int Lmax, int Lcap, float* Pt, int b,
                                             int tile) {
    constexpr int KQ = ENC_ / 4;   // k per wave
    constexpr int NG = KQ / 16;    // float4 groups per lane
    const int dt = tile % (ADIM / 16), jt = tile / (ADIM / 16);
    const int d0 = dt * 16, j0 = jt * 16;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m = lane & 15, q = lane >> 4;
    const int k0 = wave * KQ + 4 * q;
    const bool rowok = j0 + m < Lmax;
    const float4* ar = reinterpret_cast<const float4*>(enc + ((int64_t)b * Lcap + (rowok ? j0 + m : 0)) * ENC_ + k0);
    const float4* br = reinterpret_cast<const float4*>(W + (int64_t)(d0 + m) * ENC_ + k0);
    float4 a4[NG], b4[NG];
#pragma unroll
    for (int u = 0; u < NG; ++u) {
        a4[u] = ar[4 * u];
        b4[u] = br[4 * u];
    }
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NG; ++u) {
        const float4 a = rowok ? a4[u] : float4{0.f, 0.f, 0.f, 0.f};
        acc = mfma16x16x4(a.x, b4[u].x, acc);
        acc = mfma16x16x4(a.y, b4[u].y, acc);
        acc = mfma16x16x4(a.z, b4[u].z, acc);
        acc = mfma16x16x4(a.w, b4[u].w, acc);
    }
    __shared__ float red[4][256];
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][lane * 4 + r] = acc[r];
    __syncthreads();
    // element e = tid: lane e / 4 of the D layout, register e % 4: C[4 (l >> 4) + r][l & 15]
    const float v = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
    const int l = tid >> 2, r = tid & 3;
    const int j = j0 + 4 * (l >> 4) + r, d = d0 + (l & 15);
    if (j < Lmax) Pt[((int64_t)b * ADIM + d) * Lcap + j] = v;
}
template <int ENC_>
__global__ __launch_bounds__(256) void project_inputs_mfma_kernel(const float* enc, const float* W, int Lmax, int Lcap,
                                                                  float* Pt) {
    project_tile<ENC_>(enc, W, Lmax, Lcap, Pt, blockIdx.y, blockIdx.x);
}
// The projection and the decoder's per-call init as one launch (they are independent; both precede
// the decoder's first step): workgroups [0, nproj) take projection tiles, the rest the init.
template <int ENC_>
__global__ __launch_bounds__(256) void project_init_kernel(const float* enc, const float* W, int Lmax, int Lcap,
                                                           float* Pt, int ntile, int nproj, const InitArgs ia) {
    const int bid = blockIdx.x;
    if (bid < nproj) project_tile<ENC_>(enc, W, Lmax, Lcap, Pt, bid / ntile, bid % ntile);
    else decoder_init_block(ia, bid - nproj);
}

hipError_t launch_project_init(const float* enc, const float* W, int B, int Lmax, int Lcap, float* Pt, const InitArgs& ia,
                               hipStream_t s) {
    const int ntile = (ADIM / 16) * ((Lmax + 15) / 16), nproj = ntile * B;
    const dim3 grid((unsigned)(nproj + ia.B + (ia.zero ? INIT_ZERO_BLOCKS : 0)));
    hipLaunchKernelGGL(project_init_kernel<ENC>, grid, dim3(256), 0, s, enc, W, Lmax, Lcap, Pt, ntile, nproj, ia);
    return hipGetLastError();
}

hipError_t launch_project_inputs(const float* enc, const float* W, int B, int Lmax, int Lcap, float* Pt,
                                 hipStream_t s, int enc_dim) {
    static const bool valu = [] {  // measurement: TTS_PROJ_VALU=1 runs the VALU form
        const char* v = getenv("TTS_PROJ_VALU");
        return v && v[0] == '1';
    }();
    if (!valu) {
        const dim3 grid((ADIM / 16) * ((Lmax + 15) / 16), B);
        if (enc_dim == 512)
            hipLaunchKernelGGL(project_inputs_mfma_kernel<512>, grid, dim3(256), 0, s, enc, W, Lmax, Lcap, Pt);
        else if (enc_dim == 256)
            hipLaunchKernelGGL(project_inputs_mfma_kernel<256>, grid, dim3(256), 0, s, enc, W, Lmax, Lcap, Pt);
        else
            return hipErrorInvalidValue;
        return hipGetLastError();
    }
    const dim3 grid((ADIM / PJ_DG) * ((Lmax + PJ_POS - 1) / PJ_POS), B);
    if (enc_dim == 512)
        hipLaunchKernelGGL(project_inputs_kernel<512>, grid, dim3(256), 0, s, enc, W, Lmax, Lcap, Pt);
    else if (enc_dim == 256)
        hipLaunchKernelGGL(project_inputs_kernel<256>, grid, dim3(256), 0, s, enc, W, Lmax, Lcap, Pt);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// ------------------------------------------------------------------ attention step
// One workgroup of 1024 threads per sentence; thread j owns encoder position j (L <= 1024).
// The reduction area `red` holds at least one float per thread (context partials).
// (at least 256: the QE form's context reduction holds 8 parts x 512 channels)
__host__ __device__ static inline int red_stride(int Lcap) { return Lcap > 256 ? Lcap : 256; }
size_t attention_smem_bytes(int Lcap, int location) {
    size_t f = 2 * ADIM + 3 * (size_t)Lcap + ATT_WAVES * (size_t)red_stride(Lcap) + 4 * ATT_WAVES;
    if (location) f += 2 * ((size_t)Lcap + 32) + (size_t)NLOC * Lcap + ADIM * NLOC;
    f += ATT_THREADS;  // attention_kernel's fused-query partials
    return f * sizeof(float);
}

// One barrier-pair block reduction of (sum of s, max of m, argmax of y with first-index ties).
struct Red {
    float s, m, y;
    int i;
};
__device__ __forceinline__ Red block_reduce(float s, float m, float y, int i, float* scr) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        m = fmaxf(m, __shfl_xor(m, o, 64));
        const float oy = __shfl_xor(y, o, 64);
        const int oi = __shfl_xor(i, o, 64);
        if (oy > y || (oy == y && oi < i)) { y = oy; i = oi; }
    }
    if (lane == 0) {
        scr[4 * w] = s;
        scr[4 * w + 1] = m;
        scr[4 * w + 2] = y;
        reinterpret_cast<int*>(scr)[4 * w + 3] = i;
    }
    __syncthreads();
    Red r{scr[0], scr[1], scr[2], reinterpret_cast<int*>(scr)[3]};
    for (int k = 1; k < nw; ++k) {  // fixed order: deterministic
        r.s += scr[4 * k];
        r.m = fmaxf(r.m, scr[4 * k + 1]);
        const float oy = scr[4 * k + 2];
        const int oi = reinterpret_cast<int*>(scr)[4 * k + 3];
        if (oy > r.y || (oy == r.y && oi < r.i)) { r.y = oy; r.i = oi; }
    }
    __syncthreads();  // scr reusable
    return r;
}

// Block sum / max of one value over the ATT_WAVES waves: DPP wave reductions, one LDS round, the
// waves folded in order (the QE form's reductions: one cross-lane chain instead of block_reduce's
// four shuffle chains)
__device__ __forceinline__ float block_sum16(float v, float* scr) {
    v = wave_sum_dpp(v);
    if ((threadIdx.x & 63) == 0) scr[threadIdx.x >> 6] = v;
    __syncthreads();
    float r = scr[0];
#pragma unroll
    for (int k = 1; k < ATT_WAVES; ++k) r += scr[k];
    __syncthreads();
    return r;
}
__device__ __forceinline__ float block_max16(float v, float* scr) {
    v = wave_max_dpp(v);
    if ((threadIdx.x & 63) == 0) scr[threadIdx.x >> 6] = v;
    __syncthreads();
    float r = scr[0];
#pragma unroll
    for (int k = 1; k < ATT_WAVES; ++k) r = fmaxf(r, scr[k]);
    __syncthreads();
    return r;
}

// ENC_ = encoder width, HATT_ = attention-RNN width (Tacotron2: 512 / 1024; Tacotron, TacotronGST:
// 256 / 256, layers/tacotron.py:290-300).
// QE: Tacotron2's form, the energies as QE_TILES partial sums per position from query_energy_kernel
// (location term included) and the next step's location features computed at the end.
template <int ENC_, int HATT_, bool QE>
__global__ __launch_bounds__(ATT_THREADS) void attention_kernel(const AttnArgs a) {
    // QE: ATT_SPLIT workgroups per sentence (blockIdx.x = slice ks): each recomputes the weights
    // (cheap), computes 128 context channels and a quarter of the location-feature tiles; slice 0
    // writes the per-position state (into the other parity slot: the slices read the old one)
    constexpr int ASPLIT = QE ? ATT_SPLIT : 1;
    const int ks = QE ? blockIdx.x : 0;
    const int b = QE ? blockIdx.y : blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int Lc = a.Lcap;
    const int64_t row = (int64_t)b * Lc;
    constexpr int DPW = ADIM / ATT_WAVES;  // attention dims per wave in the energy loop
    // ---- phase 0: every load that depends only on kernel arguments is issued up front, so the
    // kernel pays one memory round trip before computing (latency-bound at batch 1)
    const int2 st = *reinterpret_cast<const int2*>(a.step);  // {step, n_active}
    const int par = QE ? (st.x & 1) : 0;
    const float* alpha_rd = a.alpha + (QE ? par * a.sstride : 0);
    float* alpha_wr = a.alpha + (QE ? (par ^ 1) * a.sstride : 0);
    const float* cum_rd = a.att_cum + (QE ? par * a.sstride : 0);
    float* cum_wr = a.att_cum + (QE ? (par ^ 1) * a.sstride : 0);
    const int* nidx_rd = a.nidx + (QE ? par * a.istride : 0);
    int* nidx_wr = a.nidx + (QE ? (par ^ 1) * a.istride : 0);
    const int* win_rd = a.win_idx + (QE ? par * a.istride : 0);
    int* win_wr = a.win_idx + (QE ? (par ^ 1) * a.istride : 0);
    const int L = a.lens[b];
    const int j = tid;  // this thread's encoder position
    const bool in = j < L;
    // forward attention + mask: after the mask at most (n-2)%L and [n-1, n+2] are nonzero, where
    // n = argmax(prev_alpha) was carried from the previous step; the context needs only those rows
    const bool sparse = a.forward_attn && a.forward_attn_mask;
    const int n = sparse ? nidx_rd[b] : 0;
    float u = a.forward_attn ? a.u[b] : 0.f;
    // QE + transition agent: u = sigmoid(ta([context, query])) of the previous step (:220-222),
    // evaluated here from that step's context and attention-RNN output (step 0: the initial 0.5)
    const bool ta_here = QE && a.forward_attn && a.trans_agent && st.x > 0;
    float ta_p = 0.f;
    if (ta_here) {
        if (tid < ENC_) ta_p = a.ta_w[tid] * a.ctx_prev[(int64_t)b * a.ctx_ld + tid];
        if (tid < HATT_) ta_p += a.ta_w[ENC_ + tid] * a.h_att_prev[(int64_t)b * HATT_ + tid];
    }
    const float vb = a.v_b[0];
    float qv = 0.f;
    if (tid < ADIM && !a.wqT) qv = a.q[(int64_t)b * ADIM + tid];
    else if (tid >= ADIM && tid < 2 * ADIM) qv = a.v[tid - ADIM];
    // fused query_layer (common_layers.py:179; TacotronGST): thread (d = tid % 128, slice
    // ks = tid / 128) sums k in [ks * KS, (ks + 1) * KS) of W_q[d][k] h_att[k] (coalesced rows of
    // the transposed weight, h_att a broadcast read); the 8 partials meet in LDS in slice order
    constexpr int QSL = ATT_THREADS / ADIM, KS = HATT_ / QSL;
    float qpart = 0.f;
    if (!QE && a.wqT) {
        const int d = tid & (ADIM - 1), ks = tid / ADIM;
        const float* w = a.wqT + (int64_t)ks * KS * ADIM + d;
        const float* h = a.h_att + (int64_t)b * HATT_ + ks * KS;
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int k = 0; k < KS; k += 2) {
            s0 = fmaf(w[(int64_t)k * ADIM], h[k], s0);
            s1 = fmaf(w[(int64_t)(k + 1) * ADIM], h[k + 1], s1);
        }
        qpart = s0 + s1;
    }
    const float aold_j = (a.forward_attn && in) ? alpha_rd[row + j] : 0.f;
    // Tacotron2: the energies arrive as QE_TILES partial sums per position from query_energy_kernel
    // (location term included), and this launch leaves the next step's location features
    constexpr bool qe = QE;
    float ep[QE_TILES];
#pragma unroll
    for (int k = 0; k < QE_TILES; ++k) ep[k] = (qe && in) ? a.epart[((int64_t)b * QE_TILES + k) * Lc + j] : 0.f;
    const float cum_old = (qe && a.locf && in) ? cum_rd[row + j] : 0.f;
    const float* Pt = a.Pt + (int64_t)b * ADIM * Lc;
    const int d0 = wave * DPW;
    float pv0[DPW], pv1[DPW];
#pragma unroll
    for (int dd = 0; dd < DPW; ++dd) {
        pv0[dd] = !qe && lane < L ? Pt[(int64_t)(d0 + dd) * Lc + lane] : 0.f;
        pv1[dd] = !qe && lane + 64 < L ? Pt[(int64_t)(d0 + dd) * Lc + lane + 64] : 0.f;
    }
    const float* encb = a.enc + row * ENC_;
    const int cx = sparse ? (n - 2 + L) % L : 0;
    const int clo = sparse ? (n >= 1 ? n - 1 : L - 1) : 0;
    const int chi = sparse ? min(n + 2, L - 1) : -1;
    float ex = 0.f, erow[4] = {0.f, 0.f, 0.f, 0.f};
    if (sparse && tid < ENC_) {
        ex = encb[(int64_t)cx * ENC_ + tid];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (clo + k <= chi) erow[k] = encb[(int64_t)(clo + k) * ENC_ + tid];
    }
    if (st.y == 0) return;
    const int t = st.x;
    extern __shared__ __align__(16) float sm[];
    float* q = sm;
    float* vv = q + ADIM;
    float* aold = vv + ADIM;
    float* an = aold + Lc;
    float* wts = an + Lc;
    float* red = wts + Lc;
    float* scr = red + ATT_WAVES * red_stride(Lc);
    float* cat = scr + 4 * ATT_WAVES;
    float* locf = cat + 2 * (Lc + 32);
    float* wd = locf + NLOC * Lc;

    if (!QE && a.wqT) {
        // the partials go through their own scratch at the end of the allocation; slice sums in
        // order 0..7
        float* qsc = a.location_attn ? wd + ADIM * NLOC : cat;
        qsc[tid] = qpart;
        __syncthreads();
        if (tid < ADIM) {
            float sq = 0.f;
#pragma unroll
            for (int k = 0; k < QSL; ++k) sq += qsc[k * ADIM + tid];
            qv = sq;
        }
        __syncthreads();
    }
    if (ta_here) u = sigmoidf_(block_sum16(ta_p, scr) + a.ta_b[0]);
    if (tid < ADIM) q[tid] = qv;
    else if (tid < 2 * ADIM) vv[tid - ADIM] = qv;
    if (a.forward_attn && in) aold[j] = aold_j;
    if (qe && a.locf)  // location_conv weights for the next step's features (end of this launch)
        for (int i = tid; i < NLOC * 2 * KLOC; i += blockDim.x) wd[i] = a.loc_conv[i];
    if (a.location_attn && !qe) {
        // attention_cat = [attention_weights; attention_weights_cum] (common_layers.py:167-169),
        // zero padded by (31-1)/2 = 15 on both sides for location_conv (:90-96).
        for (int c = tid; c < L + 2 * 15; c += blockDim.x) {
            const int p = c - 15;
            const bool ok = p >= 0 && p < L;
            cat[c] = ok ? a.att_w[row + p] : 0.f;
            cat[Lc + 32 + c] = ok ? a.att_cum[row + p] : 0.f;
        }
        for (int i = tid; i < ADIM * NLOC; i += blockDim.x) wd[i] = a.loc_dense[i];
    }
    __syncthreads();
    if (a.location_attn && !qe) {
        for (int idx = tid; idx < NLOC * L; idx += blockDim.x) {
            const int f = idx / L, jj = idx - f * L;
            const float* cw = a.loc_conv + f * 2 * KLOC;
            float s = 0.f;
            for (int k = 0; k < KLOC; ++k) s += cw[k] * cat[jj + k];
            for (int k = 0; k < KLOC; ++k) s += cw[KLOC + k] * cat[Lc + 32 + jj + k];
            locf[f * Lc + jj] = s;
        }
        __syncthreads();
    }
    // ---- energy partials e_j = v . tanh(pq [+ loc_j] + P_j) + b_v (common_layers.py:166-182):
    // wave w owns d in [8w, 8w+8), lanes own positions
    for (int j0 = 0; j0 < L && !qe; j0 += 64) {
        const int jj = j0 + lane;
        if (jj < L) {
            float s = 0.f;
#pragma unroll
            for (int dd = 0; dd < DPW; ++dd) {
                const int d = d0 + dd;
                float x = q[d];
                if (a.location_attn) {
                    float lc = 0.f;
                    for (int f = 0; f < NLOC; ++f) lc += wd[d * NLOC + f] * locf[f * Lc + jj];
                    x += lc;
                }
                x += j0 == 0 ? pv0[dd] : (j0 == 64 ? pv1[dd] : Pt[(int64_t)d * Lc + jj]);
                s += vv[d] * tanh_fast(x);
            }
            red[wave * Lc + jj] = s;
        }
    }
    __syncthreads();
    float e = -INFINITY;
    if (in && qe) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < QE_TILES; ++k) s += ep[k];
        e = s + vb;
    } else if (in) {
        float s = 0.f;
        for (int w = 0; w < ATT_WAVES; ++w) s += red[w * Lc + j];
        e = s + vb;
    }
    // ---- eval-mode windowing (common_layers.py:184-197)
    if (a.windowing) {
        const int wi = win_rd[b];
        const int back = wi - 2, front = wi + 6;
        if (in && ((back > 0 && j < back) || (front < L && j >= front))) e = -INFINITY;
        if (wi == -1) {
            const Red r = block_reduce(0.f, in ? e : -INFINITY, 0.f, 0, scr);
            if (j == 0) e = r.m;
        }
        const Red r = block_reduce(0.f, -INFINITY, in ? e : -INFINITY, in ? j : 0x7fffffff, scr);
        if (tid == 0 && ks == 0) win_wr[b] = r.i;
    }
    // ---- normalisation (common_layers.py:239-245)
    float al = 0.f;
    if (QE && a.attn_norm == 0) {
        const float mx = block_max16(e, scr);
        const float exj = in ? expf(e - mx) : 0.f;
        al = exj / block_sum16(exj, scr);
    } else if (QE) {
        const float sg = in ? sigmoidf_(e) : 0.f;
        al = sg / block_sum16(sg, scr);
    } else if (a.attn_norm == 0) {
        const Red r1 = block_reduce(0.f, e, 0.f, 0, scr);
        const float exj = in ? expf(e - r1.m) : 0.f;
        const Red r2 = block_reduce(exj, -INFINITY, 0.f, 0, scr);
        al = exj / r2.s;
    } else {
        const float sg = in ? sigmoidf_(e) : 0.f;
        const Red r = block_reduce(sg, -INFINITY, 0.f, 0, scr);
        al = sg / r.s;
    }
    // update_location_attention (:163-164)
    const float cum_new = cum_old + al;
    if (a.location_attn && in) {
        if (qe && a.locf) {
            if (ks == 0) cum_wr[row + j] = cum_new;
        } else {
            a.att_cum[row + j] += al;
        }
    }

    float w = al;
    if (a.forward_attn) {
        // apply_forward_attention (common_layers.py:199-223)
        float anj = 0.f;
        if (in) {
            const float prev = j ? aold[j - 1] : 0.f;
            const float mix = __fadd_rn(__fadd_rn(__fmul_rn(1.f - u, aold_j), __fmul_rn(u, prev)), 1e-8f);
            anj = __fmul_rn(mix, al);
        }
        float denom;
        if (sparse) {
            const Red r = QE ? Red{0.f, block_max16(in ? anj : -INFINITY, scr), 0.f, 0}
                             : block_reduce(0.f, in ? anj : -INFINITY, 0.f, 0, scr);
            // Python slicing of :211-213 incl. the negative-index wrap for n < 2
            if (in && ((j >= n + 3) || (n >= 1 ? j < n - 1 : j < L - 1))) anj = 0.f;
            if (j == cx) anj = 0.01f * r.m;
            if (in) an[j] = anj;
            __syncthreads();
            // the <= 5 surviving entries, summed in index order by every thread (identical result)
            denom = 0.f;
            if (cx < clo) denom += an[cx];
            for (int p = clo; p <= chi; ++p) denom += an[p];
            if (cx > chi) denom += an[cx];
        } else {
            denom = QE ? block_sum16(in ? anj : 0.f, scr) : block_reduce(in ? anj : 0.f, -INFINITY, 0.f, 0, scr).s;
        }
        w = in ? anj / denom : 0.f;
        if (in && ks == 0) alpha_wr[row + j] = w;
    }
    if (in) wts[j] = w;
    __syncthreads();
    // ---- outputs: attention weights (alpha or alignment), history, stop-rule tail (tacotron2.py:268)
    if (!QE && a.location_attn && in) a.att_w[row + j] = w;  // (QE: the features carry it)
    if (qe && a.locf) {
        // the next step's location features: location_conv over [attention_weights;
        // attention_weights_cum] = [w; cum_new] zero-padded by 15 (common_layers.py:90-104, 167-171),
        // channel 0's taps then channel 1's, the order of the launch-local evaluation
        for (int c = tid; c < L + 2 * 15; c += blockDim.x) {  // cat: [2][Lc + 32]
            const int p = c - 15;
            const bool ok = p >= 0 && p < L;
            cat[c] = ok ? wts[p] : 0.f;
        }
        if (in) cat[Lc + 32 + 15 + j] = cum_new;
        if (tid < 15) {
            cat[Lc + 32 + tid] = 0.f;
            cat[Lc + 32 + 15 + L + tid] = 0.f;
        }
        __syncthreads();  // (wd holds the conv weights [f][c][k], staged at the start)
        // as an MFMA GEMM: out[j][f] = sum_kk A[j][kk] B[kk][f], kk = 31 c + k < 62 (padded to 64),
        // A[j][kk] = cat[c][j + k] (im2col from LDS), B[kk][f] = W[f][kk]; tiles of 16 positions x
        // 16 filters, one per wave at a time, the taps in order (channel 0's, then channel 1's)
        float* lo = a.locf + (int64_t)b * NLOC * Lc;
        const int ntile = (L + 15) / 16 * 2;
        for (int tl = ks + ASPLIT * wave; tl < ntile; tl += ASPLIT * ATT_WAVES) {
            const int pt = tl >> 1, ft = tl & 1;
            const int jA = pt * 16 + (lane & 15), fB = ft * 16 + (lane & 15);
            floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s4 = 0; s4 < 16; ++s4) {
                const int kk = 4 * s4 + (lane >> 4);
                const int c = kk >= KLOC ? 1 : 0, k = kk - c * KLOC;
                const float av = kk < 2 * KLOC && jA < L ? cat[c * (Lc + 32) + jA + k] : 0.f;
                const float bv = kk < 2 * KLOC ? wd[fB * 2 * KLOC + kk] : 0.f;
                acc = mfma16x16x4(av, bv, acc);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int jj = pt * 16 + 4 * (lane >> 4) + r;
                if (jj < L) lo[(int64_t)fB * Lc + jj] = acc[r];
            }
        }
    }
    if (ks == 0 && !a.done[b] && t < a.hist_cap && a.align_hist)
        for (int jj = tid; jj < a.Lalign; jj += blockDim.x)
            a.align_hist[(int64_t)b * a.align_ldb + (int64_t)t * a.Lalign + jj] = jj < L ? wts[jj] : 0.f;
    if (tid == 0 && ks == 0) {
        a.tail[b] = a.tail_rule ? wts[L - 1] : (L >= 2 ? wts[L - 2] + wts[L - 1] : wts[0]);
        if (sparse) {
            // next step's n = argmax(prev_alpha) = 1 + first argmax of alpha[0..L-2], or 0 when
            // those are all zero; only the surviving positions can be nonzero (index order, strict >)
            float bv = 0.f;
            int bi = -1;
            auto consider = [&](int p) {
                if (p <= L - 2 && wts[p] > bv) { bv = wts[p]; bi = p; }
            };
            if (cx < clo) consider(cx);
            for (int p = clo; p <= chi; ++p) consider(p);
            if (cx > chi) consider(cx);
            nidx_wr[b] = bi >= 0 ? bi + 1 : 0;
        }
    }
    // ---- context = w . inputs  (bmm, common_layers.py:217 / 253)
    float ctx = 0.f;
    if (sparse) {
        if (tid < ENC_) {
            if (cx < clo) ctx += wts[cx] * ex;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (clo + k <= chi) ctx += wts[clo + k] * erow[k];
            if (cx > chi) ctx += wts[cx] * ex;
        }
    } else if (QE) {
        // this slice's ENC_ / ASPLIT channels as float4 groups x PARTS interleaved position sets;
        // each thread issues a batch of 8 rows' loads together (the rows stream from L2 / MALL: one
        // round trip per batch, not per row), then the parts meet in LDS and are summed in order
        constexpr int CS = ENC_ / ASPLIT, D4 = CS / 4, PARTS = ATT_THREADS / D4;
        static_assert(PARTS * CS <= ATT_WAVES * 256, "context partials fit the reduction area");
        const int d4 = ks * D4 + tid % D4, part = tid / D4;
        float4 acc = float4{0.f, 0.f, 0.f, 0.f};
        for (int j0 = part; j0 < L; j0 += 8 * PARTS) {
            float4 ev[8];
#pragma unroll
            for (int m = 0; m < 8; ++m)
                ev[m] = *reinterpret_cast<const float4*>(encb + (int64_t)min(j0 + m * PARTS, L - 1) * ENC_ + 4 * d4);
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const float wv = j0 + m * PARTS < L ? wts[j0 + m * PARTS] : 0.f;
                acc.x += wv * ev[m].x;
                acc.y += wv * ev[m].y;
                acc.z += wv * ev[m].z;
                acc.w += wv * ev[m].w;
            }
        }
        *reinterpret_cast<float4*>(red + part * CS + 4 * (tid % D4)) = acc;
        __syncthreads();
        if (tid < CS) {
            ctx = red[tid];
#pragma unroll
            for (int p = 1; p < PARTS; ++p) ctx += red[p * CS + tid];
        }
    } else {
        // PARTS interleaved position sets per channel, summed in part order
        constexpr int PARTS = ATT_THREADS / ENC_;
        const int d = tid % ENC_, part = tid / ENC_;
        float acc = 0.f;
        int jj = part;
        for (; jj + 3 * PARTS < L; jj += 4 * PARTS) {
            const float e0 = encb[(int64_t)jj * ENC_ + d];
            const float e1 = encb[(int64_t)(jj + PARTS) * ENC_ + d];
            const float e2 = encb[(int64_t)(jj + 2 * PARTS) * ENC_ + d];
            const float e3 = encb[(int64_t)(jj + 3 * PARTS) * ENC_ + d];
            acc += wts[jj] * e0;
            acc += wts[jj + PARTS] * e1;
            acc += wts[jj + 2 * PARTS] * e2;
            acc += wts[jj + 3 * PARTS] * e3;
        }
        for (; jj < L; jj += PARTS) acc += wts[jj] * encb[(int64_t)jj * ENC_ + d];
        red[tid] = acc;
        __syncthreads();
        if (tid < ENC_) {
            ctx = red[tid];
#pragma unroll
            for (int p = 1; p < PARTS; ++p) ctx += red[p * ENC_ + tid];
        }
    }
    if (QE) {  // this slice's channels (sparse: every slice evaluated all of them, cheaply)
        constexpr int CS = ENC_ / ASPLIT;
        const int dch = sparse ? tid : ks * CS + tid;
        if (sparse ? (tid >= ks * CS && tid < (ks + 1) * CS) : tid < CS) {
            a.ctx[(int64_t)b * a.ctx_ld + dch] = ctx;
            if (a.ctxf) a.ctxf[frag_idx(b, a.ctxf_k0 + dch, a.ntf)] = ctx;
        }
    } else if (tid < ENC_) {
        a.ctx[(int64_t)b * a.ctx_ld + tid] = ctx;
        if (a.ctxf) a.ctxf[frag_idx(b, a.ctxf_k0 + tid, a.ntf)] = ctx;
    }
    if (!QE && a.forward_attn && a.trans_agent) {  // (QE: at the start of the next step's launch)
        // u = sigmoid(ta([context, query]))  (:220-222)
        const float* h = a.h_att + (int64_t)b * HATT_;
        float p = tid < ENC_ ? a.ta_w[tid] * ctx : 0.f;
        if (tid < HATT_) p += a.ta_w[ENC_ + tid] * h[tid];
        const float ts = QE ? block_sum16(p, scr) : block_reduce(p, -INFINITY, 0.f, 0, scr).s;
        if (tid == 0) a.u[b] = sigmoidf_(ts + a.ta_b[0]);
    }
}

// Latency path for the synthesis configuration (synthesize.py:86): forward attention with the
// eval mask and sigmoid normalisation, no location features, no windowing, no transition agent.
// Same results as attention_kernel up to fp32 rounding, with one barrier instead of nine:
//   - the energies arrive as 8 partial sums per position from query_energy_kernel (the 128 tanh
//     per position run on 8 compute units in the query launch, not on this one);
//     prev_alpha[j] and prev_alpha[j-1] come straight from global memory;
//   - the sigmoid normaliser cancels in the forward-attention renormalisation
//     (alpha = m*s/S / sum(m*s/S)), so it is not reduced;
//   - one block reduction gives both max(alpha) (for the 0.01*val entry) and the sum of the
//     surviving window [n-1, n+2]; every thread then knows the <= 5 nonzero weights (read from
//     LDS after that reduction's barrier), so the context, the tail, the next argmax and the
//     outputs need no further synchronisation.
__global__ __launch_bounds__(ATT_THREADS) void attention_fm_kernel(const AttnArgs a) {
    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int Lc = a.Lcap;
    const int64_t row = (int64_t)b * Lc;
    // ---- phase 0: loads that depend only on the arguments
    int st_x = a.step[0], st_y = a.step[1];
    const int L = a.lens[b];
    const int n = a.nidx[b];
    const float u = a.u[b];
    const float vb = a.v_b[0];
    const int done = a.done[b];
    const int j = tid;
    const bool in = j < L;
    float ep[QE_TILES];
#pragma unroll
    for (int k = 0; k < QE_TILES; ++k) ep[k] = j < Lc ? a.epart[((int64_t)b * QE_TILES + k) * Lc + j] : 0.f;
    const float aold_j = in ? a.alpha[row + j] : 0.f;
    const float aold_p = (in && j > 0) ? a.alpha[row + j - 1] : 0.f;
    // the surviving positions after the mask: (n-2) mod L and [n-1, n+2] (Python slicing of
    // common_layers.py:211-213, including the negative-index wrap for n < 2)
    const int cx = (n - 2 + L) % L;
    const int clo = n >= 1 ? n - 1 : L - 1;
    const int chi = min(n + 2, L - 1);
    const float* encb = a.enc + row * ENC;
    float ex = 0.f, erow[4] = {0.f, 0.f, 0.f, 0.f};
    if (tid < ENC) {
        ex = encb[(int64_t)cx * ENC + tid];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (clo + k <= chi) erow[k] = encb[(int64_t)(clo + k) * ENC + tid];
    }
    extern __shared__ __align__(16) float sm[];
    float* an = sm;         // [Lc] unnormalised forward weights
    float* scr = an + Lc;   // [2 * ATT_WAVES]
    asm volatile("" : "+v"(st_x), "+v"(st_y));
    if (st_y == 0) return;  // every sentence done (uniform)
    const int t = st_x;
    // ---- energy (partials from query_energy_kernel), sigmoid, forward mix, mask
    // (common_layers.py:178-182, 199-213, 241-243)
    float anj = 0.f;
    if (in) {
        float e = 0.f;
#pragma unroll
        for (int k = 0; k < QE_TILES; ++k) e += ep[k];
        const float sg = sigmoidf_(e + vb);
        const float mix = __fadd_rn(__fadd_rn(__fmul_rn(1.f - u, aold_j), __fmul_rn(u, aold_p)), 1e-8f);
        anj = __fmul_rn(mix, sg);
        an[j] = anj;
    }
    const bool win = in && j >= clo && j <= chi && j != cx;
    // one barrier: DPP wave reductions, then every thread folds the 16 wave results in order
    const float ws = wave_sum_dpp(win ? anj : 0.f);
    const float wm = wave_max_dpp(in ? anj : -INFINITY);
    if (lane == 0) {
        scr[2 * wave] = ws;
        scr[2 * wave + 1] = wm;
    }
    __syncthreads();
    float rs = 0.f, rm = -INFINITY;
    for (int k = 0; k < ATT_WAVES; ++k) {
        rs += scr[2 * k];
        rm = fmaxf(rm, scr[2 * k + 1]);
    }
    const float vx = 0.01f * rm;  // alpha[(n-2)] = 0.01 * val
    const float denom = rs + vx;
    auto weight = [&](int p) -> float {  // normalised weight of position p (0 outside the survivors)
        if (p == cx) return vx / denom;
        return (p >= clo && p <= chi) ? an[p] / denom : 0.f;
    };
    const float w = in ? weight(j) : 0.f;
    if (in) a.alpha[row + j] = w;
    if (!done && t < a.hist_cap && a.align_hist && j < a.Lalign)
        a.align_hist[(int64_t)b * a.align_ldb + (int64_t)t * a.Lalign + j] = w;
    if (tid == 0) {
        a.tail[b] = L >= 2 ? weight(L - 2) + weight(L - 1) : weight(0);  // tacotron2.py:268
        // next step's n = argmax(prev_alpha) = 1 + first argmax of alpha[0..L-2] (0 if all zero)
        float bv = 0.f;
        int bi = -1;
        auto consider = [&](int p) {
            const float wp = weight(p);
            if (p <= L - 2 && wp > bv) { bv = wp; bi = p; }
        };
        if (cx < clo) consider(cx);
        for (int p = clo; p <= chi; ++p) consider(p);
        if (cx > chi) consider(cx);
        a.nidx[b] = bi >= 0 ? bi + 1 : 0;
    }
    // ---- context over the survivors, in index order (bmm, common_layers.py:217)
    if (tid < ENC) {
        float ctx = 0.f;
        if (cx < clo) ctx += weight(cx) * ex;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (clo + k <= chi) ctx += weight(clo + k) * (clo + k == cx ? ex : erow[k]);
        if (cx > chi) ctx += weight(cx) * ex;
        a.ctx[(int64_t)b * XA + tid] = ctx;
        if (a.ctxf) a.ctxf[frag_idx(b, a.ctxf_k0 + tid, a.ntf)] = ctx;
    }
}

static bool attention_fast(const AttnArgs& a) {
    return a.enc_dim == ENC && a.forward_attn && a.forward_attn_mask && a.attn_norm == 1 && !a.location_attn &&
           !a.windowing && !a.trans_agent;
}
bool attention_uses_epart(const AttnArgs& a) { return attention_fast(a); }

// ------------------------------------------------------------------ query + energy partials
__global__ __launch_bounds__(1024) void query_energy_kernel(const QEArgs a) {
    const int tile = blockIdx.x, b = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int Lc = a.Lcap;
    constexpr int NCH = HATT / 16;      // k-chunks of 16
    constexpr int CPW = NCH / 16;       // chunks per wave (16 waves)
    // ---- phase 0: weights, activations, P rows of this thread's position, v, step state
    int st_y = a.step[1];
    const int L = a.lens[b];
    const int j = tid;
    float pt[16];
    const float* Pt = a.Pt + ((int64_t)b * ADIM + tile * 16) * Lc;
#pragma unroll
    for (int dd = 0; dd < 16; ++dd) pt[dd] = (a.energies && j < Lc) ? Pt[(int64_t)dd * Lc + j] : 0.f;
    // this tile's 16 rows of location_dense (LDS, [d][f] padded against bank conflicts)
    __shared__ float wld[16][NLOC + 1];
    const bool loc = a.energies && a.locf;
    if (loc && tid < 16 * NLOC) wld[tid / NLOC][tid % NLOC] = a.loc_dense[(tile * 16 + tid / NLOC) * NLOC + tid % NLOC];
    const float4* Wp = reinterpret_cast<const float4*>(a.Wq) + ((size_t)tile * NCH + wave * CPW) * 64 + lane;
    const float* hb = a.h + (int64_t)b * HATT + (lane >> 4) * 4;
    float4 wv[CPW], xv[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        wv[c] = Wp[(size_t)c * 64];
        xv[c] = *reinterpret_cast<const float4*>(hb + (wave * CPW + c) * 16);
    }
    float acc = 0.f, acc2 = 0.f;
#pragma unroll
    for (int c = 0; c < CPW; c += 2) {
        acc = fmaf(wv[c].x, xv[c].x, acc);
        acc = fmaf(wv[c].y, xv[c].y, acc);
        acc = fmaf(wv[c].z, xv[c].z, acc);
        acc = fmaf(wv[c].w, xv[c].w, acc);
        acc2 = fmaf(wv[c + 1].x, xv[c + 1].x, acc2);
        acc2 = fmaf(wv[c + 1].y, xv[c + 1].y, acc2);
        acc2 = fmaf(wv[c + 1].z, xv[c + 1].z, acc2);
        acc2 = fmaf(wv[c + 1].w, xv[c + 1].w, acc2);
    }
    float s = acc + acc2;
    s += __shfl_xor(s, 16, 64);  // the four k-groups of row (lane & 15)
    s += __shfl_xor(s, 32, 64);
    asm volatile("" : "+v"(st_y));
    if (st_y == 0) return;  // every sentence done (uniform)
    __shared__ float red[16][16];
    __shared__ float qs[16];
    if (lane < 16) red[wave][lane] = s;
    __syncthreads();
    if (tid < 16) {
        float q = 0.f;
        for (int w = 0; w < 16; ++w) q += red[w][tid];  // fixed order: deterministic
        qs[tid] = q;
        a.q[(int64_t)b * ADIM + tile * 16 + tid] = q;
    }
    if (!a.energies) return;
    __syncthreads();
    if (loc) {
        // get_location_attention (common_layers.py:166-176): tanh(processed_query +
        // location_dense(location_conv(attention_cat)) + processed_inputs), summed in that order.
        // location_dense as an MFMA GEMM per 16 positions: C[j][d] = sum_f locf[f][j] W[d][f]
        // (lane: positions j0 + 4 (lane >> 4) + r, dim lane & 15), then the 16 dims' v . tanh
        // summed across each 16-lane row
        const int d = lane & 15;
        const float vd = a.v[tile * 16 + d], qd = qs[d];
        const float* lp = a.locf + (int64_t)b * NLOC * Lc;
        const float* Pd = a.Pt + ((int64_t)b * ADIM + tile * 16 + d) * Lc;
        for (int j0 = wave * 16; j0 < L; j0 += 16 * 16) {
            floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
            const int jA = min(j0 + (lane & 15), L - 1);
#pragma unroll
            for (int s4 = 0; s4 < NLOC / 4; ++s4) {
                const int f = 4 * s4 + (lane >> 4);
                acc = mfma16x16x4(lp[(int64_t)f * Lc + jA], wld[d][f], acc);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int jj = j0 + 4 * (lane >> 4) + r;
                float e = vd * tanh_fast((qd + acc[r]) + Pd[min(jj, L - 1)]);
                e += __shfl_xor(e, 1, 64);
                e += __shfl_xor(e, 2, 64);
                e += __shfl_xor(e, 4, 64);
                e += __shfl_xor(e, 8, 64);
                if (d == 0 && jj < L) a.epart[((int64_t)b * QE_TILES + tile) * Lc + jj] = e;
            }
        }
    } else if (j < L) {
        float e = 0.f;
#pragma unroll
        for (int dd = 0; dd < 16; ++dd) e += a.v[tile * 16 + dd] * tanh_fast(qs[dd] + pt[dd]);
        a.epart[((int64_t)b * QE_TILES + tile) * Lc + j] = e;
    }
}

hipError_t launch_query_energy(const QEArgs& a, int B, hipStream_t s) {
    hipLaunchKernelGGL(query_energy_kernel, dim3(QE_TILES, B), dim3(1024), 0, s, a);
    return hipGetLastError();
}

static size_t attention_fm_smem_bytes(int Lcap) {
    return ((size_t)Lcap + 2 * ATT_WAVES) * sizeof(float);
}

__global__ void transpose_f32_kernel(const float* src, int rows, int cols, float* dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)rows * cols) return;
    const int r = (int)(i / cols), c = (int)(i % cols);
    dst[(int64_t)c * rows + r] = src[i];
}

hipError_t transpose_f32(const float* src, int rows, int cols, float* dst, hipStream_t s) {
    const int64_t n = (int64_t)rows * cols;
    hipLaunchKernelGGL(transpose_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, rows, cols, dst);
    return hipGetLastError();
}

hipError_t launch_attention(const AttnArgs& a, hipStream_t s) {
    if (attention_fast(a)) {
        hipLaunchKernelGGL(attention_fm_kernel, dim3(a.B), dim3(ATT_THREADS), attention_fm_smem_bytes(a.Lcap), s, a);
    } else if (a.enc_dim == ENC && a.epart) {
        hipLaunchKernelGGL((attention_kernel<ENC, HATT, true>), dim3(ATT_SPLIT, a.B), dim3(ATT_THREADS),
                           attention_smem_bytes(a.Lcap, a.location_attn), s, a);
    } else if (a.enc_dim == ENC) {
        hipLaunchKernelGGL((attention_kernel<ENC, HATT, false>), dim3(a.B), dim3(ATT_THREADS),
                           attention_smem_bytes(a.Lcap, a.location_attn), s, a);
    } else if (a.enc_dim == 256) {
        hipLaunchKernelGGL((attention_kernel<256, 256, false>), dim3(a.B), dim3(ATT_THREADS),
                           attention_smem_bytes(a.Lcap, a.location_attn), s, a);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t attention_prepare(int Lcap, int location) {
    const int bytes = (int)attention_smem_bytes(Lcap, location);
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_kernel<ENC, HATT, true>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_kernel<ENC, HATT, false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_kernel<256, 256, false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_fm_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)attention_fm_smem_bytes(Lcap));
}

}  // namespace tts

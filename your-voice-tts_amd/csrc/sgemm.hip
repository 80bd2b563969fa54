// Skinny fp32 MFMA GEMM + fused LSTM cell epilogue (see sgemm.h for the layout).
//
// Replaces, per decoder step (layers/tacotron2.py:194-224, common_layers.py:77-83,170):
//   attention_rnn / decoder_rnn  nn.LSTMCell  (gates GEMV + pointwise, fused here)
//   prenet linear+relu, query_layer, linear_projection.
// Roofline at small batch: HBM/Infinity-Cache bound on the weight stream (each packed weight
// byte is read exactly once per step by exactly one wave) and launch latency; at batch 64 the
// gate GEMMs approach the fp32 MFMA bound (dec_lstm 1.34 GFLOP: 8.5 us at 157 TF; measured 15.5).
#include <cstdlib>

#include "sgemm.h"

namespace tts {

constexpr int MAX_WAVES = 16;
#ifndef TTS_NT_ROLES
#define TTS_NT_ROLES 0
#endif
constexpr int PRE_DIM = 256;  // prenet width (layers/tacotron2.py:108)
__device__ const int kOneActive[2] = {0, 1};  // {step 0, 1 active} for launches without step state

// Activation addressing of one lane: segments p0 | p1 | p2 of the concatenated row (wave-uniform
// bases shifted by each segment's first chunk, row strides, first chunk past segments 0 and 1,
// floats per chunk) and the lane's rows (one per m-tile) and offset.  Element (m-tile mt, chunk
// c) of the lane = p_s + c * cs + xk + row[mt] * ld_s.  Row-major activations: cs = 16, xk = the
// lane's k offset, row = the batch row.  Fragment mirrors (Seg::pf): cs = ntf * 256, ld = 1,
// xk = 4 * lane, row = 256 * m-tile.
template <int NT>
struct XAddr {
    const float *p0 = nullptr, *p1 = nullptr, *p2 = nullptr;
    int ld0 = 0, ld1 = 0, ld2 = 0, cb0 = 0, cb1 = 0;
    int cs = 16;
    int row[NT];
    int xk = 0;
};

// One pipeline stage: the weight fragment and the NT activation fragments of chunks
// [c0, c0 + UP).  Chunks past cend load chunk cend-1 again (callers skip their FMAs): every load
// is unconditional, so the wait before a stage's MFMAs counts exactly the next stage's loads
// (a load under a branch makes the compiler wait for everything).  Requires cend > c0.
template <int UP, int NT, int ROLE, bool FRAG = false>
__device__ __forceinline__ void sg_load(const float4* __restrict__ Wp, const XAddr<NT> xa, int c0, int cend,
                                        float4 (&wv)[UP], float4 (&xv)[UP][NT]) {
#pragma unroll
    for (int u = 0; u < UP; ++u) {
        const int c = min(c0 + u, cend - 1);
        if ((TTS_NT_ROLES >> ROLE) & 1) {
            // non-temporal (stream) policy: this matrix passes through L2 without evicting the
            // default-policy matrices that stay resident there across steps
            const floatx4 t = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(Wp + (size_t)c * 64));
            wv[u] = float4{t[0], t[1], t[2], t[3]};
        } else {
            wv[u] = Wp[(size_t)c * 64];
        }
        // wave-uniform segment: scalar base + c * cs and row stride, per-lane row and offset
        const bool s0 = c < xa.cb0, s1 = c < xa.cb1;
        const float* base = (s0 ? xa.p0 : (s1 ? xa.p1 : xa.p2)) + c * xa.cs + xa.xk;
        if (FRAG) {
            // uniform chunk base + a 32-bit per-lane offset: the load's scalar-base form, no
            // per-load 64-bit address arithmetic
            const float* cbase = (s0 ? xa.p0 : (s1 ? xa.p1 : xa.p2)) + c * xa.cs;
#pragma unroll
            for (int mt = 0; mt < NT; ++mt)
                xv[u][mt] = *reinterpret_cast<const float4*>(cbase + (unsigned)(xa.row[mt] + xa.xk));
        } else {
            const int ld = s0 ? xa.ld0 : (s1 ? xa.ld1 : xa.ld2);
#pragma unroll
            for (int mt = 0; mt < NT; ++mt) xv[u][mt] = *reinterpret_cast<const float4*>(base + xa.row[mt] * ld);
        }
    }
}

// The MFMAs of one stage; chunk u accumulates into chain u & 1 at NT == 1 (two independent
// chains hide the MFMA latency), into the m-tile's one chain otherwise (NT chains interleave).
// Padding chunks (past cend: sg_load re-loaded chunk cend-1) multiply a zeroed weight fragment:
// no branch around an MFMA, so the accumulators need no copies between loop blocks (copies that
// otherwise force a full memory wait ahead of the next stage's loads).
template <int UP, int NT>
__device__ __forceinline__ void sg_mfma(int c0, int cend, const float4 (&wv)[UP], const float4 (&xv)[UP][NT],
                                        floatx4 (&acc)[2][NT]) {
#pragma unroll
    for (int u = 0; u < UP; ++u) {
        const bool live = c0 + u < cend;  // wave-uniform
        const float4 w = live ? wv[u] : float4{0.f, 0.f, 0.f, 0.f};
        const int ch = NT == 1 ? (u & 1) : 0;
#pragma unroll
        for (int mt = 0; mt < NT; ++mt) acc[ch][mt] = mfma16x16x4(xv[u][mt].x, w.x, acc[ch][mt]);
#pragma unroll
        for (int mt = 0; mt < NT; ++mt) acc[ch][mt] = mfma16x16x4(xv[u][mt].y, w.y, acc[ch][mt]);
#pragma unroll
        for (int mt = 0; mt < NT; ++mt) acc[ch][mt] = mfma16x16x4(xv[u][mt].z, w.z, acc[ch][mt]);
#pragma unroll
        for (int mt = 0; mt < NT; ++mt) acc[ch][mt] = mfma16x16x4(xv[u][mt].w, w.w, acc[ch][mt]);
    }
}

// ROLE only names the instantiation (distinct kernel names in rocprof traces per decoder stage).
// MT = m-tiles of 16 batch rows on the MFMA path; MT = 0 is the batch-1 VALU path.  FRAG: the
// activations come from fragment mirrors (Seg::pf) and the workgroup is 4 waves, one per SIMD
// (sgemm_frag_kernel); otherwise 16 waves read row-major activations (sgemm_kernel).
template <int MT, int EPI, int ROLE, bool FRAG>
__device__ __forceinline__ void sgemm_body(const SGemmArgs& a) {
    constexpr bool VALU = MT == 0;
    constexpr int NT = VALU ? 1 : MT;
    // Latency structure (batch-1 decode: every launch is one dependent link of the step chain):
    // the step state, the epilogue operands, and the wave's whole weight + activation slice are
    // all issued as vector loads before anything waits, so a launch pays one memory round trip.
    // (A scalar load of the step state would be waited on at once, before the weight loads
    // issue.)  The "all sentences done" exit is taken after the MFMAs: it only costs steps past
    // the end.
    // a global-address-space load: through a generic pointer this would be a FLAT load, which
    // counts in both vmcnt and lgkmcnt and makes every later memory wait of the main loop a full one
    typedef const __attribute__((address_space(1))) int* gint_p;
    const gint_p sp = (gint_p)(a.step ? a.step : kOneActive);
    int st_x = sp[0];
    int st_y = sp[1];
    const int ntile = blockIdx.x;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar loop control
    const int nw = blockDim.x >> 6;
    const int tid = threadIdx.x;
    // row group: this workgroup's batch rows [m0, m0 + Bh) (grid.y > 1 splits the batch over
    // workgroups, sgemm_launch)
    const int m0 = blockIdx.y * 16 * NT;
    const int Bh = min(a.B - m0, 16 * NT);
    float pre_bias[4] = {0.f, 0.f, 0.f, 0.f}, pre_cell = 0.f;
    int pre_done = 0;
    if ((EPI == EPI_LINEAR || EPI == EPI_MEL_FUSED) && tid < Bh * 16) {
        const int n = ntile * 16 + (tid & 15);
        if (a.bias && n < a.N) pre_bias[0] = a.bias[n];
        if (a.done) pre_done = a.done[m0 + (tid >> 4)];
    }
    // stop-rule operands of the fused mel launch (one workgroup per row group, one thread per
    // sentence)
    const int stop_tile = EPI == EPI_MEL_FUSED ? (a.mf.nmel + PRE_DIM) >> 4 : -1;
    int sr_done = 1, sr_len = 0, sr_flag = 0, sr_count = 0;
    float sr_tail = 0.f, sr_bias = 0.f;
    if (EPI == EPI_MEL_FUSED && ntile == stop_tile && tid < Bh) {
        sr_done = a.done[m0 + tid];
        sr_len = a.mf.lens[m0 + tid];
        sr_flag = a.mf.flag1[m0 + tid];
        sr_count = a.mf.count[m0 + tid];
        sr_tail = a.mf.tail[m0 + tid];
        // lane-dependent index (B <= 64, so tid & (B >> 8) == 0): a vector load, waited late,
        // not a scalar one waited at the next kernel-argument load
        sr_bias = a.bias[a.mf.nmel + PRE_DIM + (tid & (a.B >> 8))];
    }
    if (EPI == EPI_LSTM && tid < Bh * 4) {
        const int b = m0 + (threadIdx.x >> 2), u = threadIdx.x & 3;
#pragma unroll
        for (int g = 0; g < 4; ++g) pre_bias[g] = a.bias[ntile * 16 + g * 4 + u];
        pre_cell = a.cell[(int64_t)b * a.ldc + ntile * 4 + u];
    }
    float pre_res = 0.f;  // EPI_GRU: residual input of this (sentence, unit)
    if (EPI == EPI_GRU && tid < Bh * 4) {
        const int b = m0 + (threadIdx.x >> 2), u = threadIdx.x & 3;
#pragma unroll
        for (int g = 0; g < 4; ++g) pre_bias[g] = a.bias[ntile * 16 + g * 4 + u];
        pre_cell = a.gru.h[(int64_t)b * a.gru.ldh + ntile * 4 + u];  // h_{t-1}
        if (a.gru.res) pre_res = a.gru.res[(int64_t)b * a.gru.ldr + ntile * 4 + u];
    }
    const int dir = EPI == EPI_ENC_LSTM ? ntile / a.enc.tiles_per_dir : 0;
    int enc_pos = -1;  // encoder position this thread's (b, unit) updates, -1 when idle
    if (EPI == EPI_ENC_LSTM && (int)threadIdx.x < Bh * 4) {
        const EncLstm& E = a.enc;
        const int b = m0 + (threadIdx.x >> 2), u = threadIdx.x & 3;
        const int unit = (ntile - dir * E.tiles_per_dir) * 4 + u;
        const int L = E.lens[b];
        if (E.s < L) {
            enc_pos = dir ? L - 1 - E.s : E.s;
            const float* xi = E.xi + ((int64_t)b * E.Tmax + enc_pos) * (8 * E.H) + dir * 4 * E.H + unit;
#pragma unroll
            for (int g = 0; g < 4; ++g) pre_bias[g] = xi[g * E.H];
            pre_cell = E.c[dir * E.cstride + (int64_t)b * E.H + unit];
        }
    }
    const int nchunks = a.K >> 4;
    const int cbeg = wave * nchunks / nw;
    const int cend = (wave + 1) * nchunks / nw;

    // Activation addressing (XAddr): a wave-uniform base and stride per segment, per lane the
    // row b = m0 + mt*16 + (lane&15) of each m-tile (VALU path: row 0 for every lane) and the k
    // offset (lane>>4)*4.  Rows past the batch read row B-1 instead: an MFMA output row depends
    // on its own input row only, and the epilogue never stores rows >= B.
    const int xrow = VALU ? 0 : lane & 15;
    const int xk = (lane >> 4) * 4;
    XAddr<NT> xa;
    int kstart = 0;
    const int fcs = FRAG ? a.ntf * 256 : 16;  // floats per chunk
#pragma unroll
    for (int s = 0; s < 3; ++s) {
        // the encoder LSTM reads one segment: its direction's previous hidden state
        const Seg& g = a.seg[EPI == EPI_ENC_LSTM ? (s == 0 ? dir : 2) : s];
        const bool live = EPI == EPI_ENC_LSTM ? s == 0 : s < a.nseg;
        const float* base = live ? (FRAG ? g.pf : g.p) - (kstart >> 4) * fcs : nullptr;
        const int ld = live ? (FRAG ? 1 : g.ld) : 0;
        kstart += live ? g.len : 0;
        if (s == 0) { xa.p0 = base; xa.ld0 = ld; xa.cb0 = kstart >> 4; }
        if (s == 1) { xa.p1 = base; xa.ld1 = ld; xa.cb1 = kstart >> 4; }
        if (s == 2) { xa.p2 = base; xa.ld2 = ld; }
    }
    xa.cs = fcs;
#pragma unroll
    for (int mt = 0; mt < NT; ++mt) xa.row[mt] = FRAG ? ((m0 >> 4) + mt) * 256 : min(m0 + mt * 16 + xrow, a.B - 1);
    xa.xk = FRAG ? 4 * lane : xk;

    floatx4 acc[2][NT];  // MFMA accumulators (see sg_mfma)
#pragma unroll
    for (int mt = 0; mt < NT; ++mt) acc[0][mt] = acc[1][mt] = floatx4{0.f, 0.f, 0.f, 0.f};
    float vacc = 0.f, vacc2 = 0.f;  // VALU path

    const float4* __restrict__ Wp = reinterpret_cast<const float4*>(a.W) + (size_t)ntile * nchunks * 64 + lane;
    if (!VALU) {
        // Two register stages of UP chunks: the loads of stage s+1 are in flight while stage s
        // runs its MFMAs (one memory round trip exposed per wave, not one per stage).  Row-major
        // at batch <= 16: 16 waves, one stage of 4 covers most of a wave's chunks; over mirrors
        // at batch 64: 4 waves, a wave owns 40 chunks of the widest GEMM, 20 stages of 2.
        constexpr int UP = (NT == 1 && !FRAG) ? 4 : 2;
        float4 wA[UP], xA[UP][NT], wB[UP], xB[UP][NT];
        // (the scheduling barriers keep each stage's loads issued ahead of the previous stage's
        // MFMAs: left alone the scheduler sinks them below, which serialises load and MFMA time)
        // Stage pairs without an exit in between (a mid-loop exit makes the register allocator
        // rotate the accumulators through copies at the back edge); an odd last stage runs after
        // the loop on the loads its last iteration issued.
        const int nst = (cend - cbeg + UP - 1) / UP;
        if (nst > 0) sg_load<UP, NT, ROLE, FRAG>(Wp, xa, cbeg, cend, wA, xA);
        int st = 0;
        for (; st + 1 < nst; st += 2) {
            const int c0 = cbeg + st * UP;
            sg_load<UP, NT, ROLE, FRAG>(Wp, xa, c0 + UP, cend, wB, xB);
            __builtin_amdgcn_sched_barrier(0);
            sg_mfma<UP, NT>(c0, cend, wA, xA, acc);
            sg_load<UP, NT, ROLE, FRAG>(Wp, xa, c0 + 2 * UP, cend, wA, xA);
            __builtin_amdgcn_sched_barrier(0);
            sg_mfma<UP, NT>(c0 + UP, cend, wB, xB, acc);
        }
        if (st < nst) sg_mfma<UP, NT>(cbeg + st * UP, cend, wA, xA, acc);
    }
    // VALU path (batch 1): U chunks of loads (U KiB of weights per wave) in flight before the
    // first FMA; one round covers every decoder shape (<= 10 chunks per wave at 16 waves, K <= 2560)
    constexpr int U = 10;
    for (int c0 = cbeg; VALU && c0 < cend; c0 += U) {
        float4 wv[U];
        float4 xv[U][NT];
        sg_load<U, NT, ROLE>(Wp, xa, c0, cend, wv, xv);
        // lane (row n = lane&15, k-group lane>>4) dots its 4 weights with x; the MFMA path would
        // pad the batch to 16 rows and pay 16x the multiplies
#pragma unroll
        for (int u = 0; u < U; u += 2) {
            if (c0 + u < cend) {
                vacc = fmaf(wv[u].x, xv[u][0].x, vacc);
                vacc = fmaf(wv[u].y, xv[u][0].y, vacc);
                vacc = fmaf(wv[u].z, xv[u][0].z, vacc);
                vacc = fmaf(wv[u].w, xv[u][0].w, vacc);
            }
            if (c0 + u + 1 < cend) {
                vacc2 = fmaf(wv[u + 1].x, xv[u + 1][0].x, vacc2);
                vacc2 = fmaf(wv[u + 1].y, xv[u + 1][0].y, vacc2);
                vacc2 = fmaf(wv[u + 1].z, xv[u + 1][0].z, vacc2);
                vacc2 = fmaf(wv[u + 1].w, xv[u + 1][0].w, vacc2);
            }
        }
    }
    if (VALU) {
        // sum the four k-groups (lanes n, n+16, n+32, n+48), then place row n's partial where the
        // MFMA accumulator fragment keeps C[b=0][n] (lane n, component 0)
        float v = vacc + vacc2;
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        acc[0][0] = floatx4{lane < 16 ? v : 0.f, 0.f, 0.f, 0.f};
    } else if (NT == 1) {
        acc[0][0] += acc[1][0];
    }

    // Operands loaded in the prologue are consumed only from here on; the empty asm redefines
    // them here so the compiler cannot hoist their first use (and its wait) above the loads.
    asm volatile("" : "+v"(st_x), "+v"(st_y), "+v"(pre_done), "+v"(pre_bias[0]), "+v"(pre_bias[1]),
                 "+v"(pre_bias[2]), "+v"(pre_bias[3]), "+v"(pre_cell), "+v"(pre_res));
    if (st_y == 0) {
        // every sentence is done: steps past the end are no-ops, but the fused stop launch
        // still forwards {step+1, 0} so the next parity slot reads "done" as well
        if (EPI == EPI_MEL_FUSED && ntile == 0 && blockIdx.y == 0 && tid == 0)
            *reinterpret_cast<int2*>(a.mf.state_next) = make_int2(st_x + 1, 0);
        return;
    }
    const int step = st_x;

    // Cross-wave K reduction in a fixed order.
    __shared__ float red[MAX_WAVES][NT][64][4];
    __shared__ float fin[NT * 16][17];
#pragma unroll
    for (int mt = 0; mt < NT; ++mt) {
        red[wave][mt][lane][0] = acc[0][mt].x;
        red[wave][mt][lane][1] = acc[0][mt].y;
        red[wave][mt][lane][2] = acc[0][mt].z;
        red[wave][mt][lane][3] = acc[0][mt].w;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < NT * 256; e += blockDim.x) {
        const int mt = e >> 8, l = (e >> 2) & 63, r = e & 3;
        float s = 0.f;
        for (int w = 0; w < nw; ++w) s += red[w][mt][l][r];
        fin[mt * 16 + (l >> 4) * 4 + r][l & 15] = s;
    }
    __syncthreads();

    const bool track = a.hist != nullptr && step < a.hist_cap;
    if (EPI == EPI_LINEAR) {
        float* out = a.out ? a.out + (a.out_par >= 0 ? (int64_t)((step + a.out_par) & 1) * a.out_pstride : 0) : nullptr;
        if (tid < Bh * 16) {  // B <= 64: one element per thread
            const int bl = tid >> 4, col = tid & 15, b = m0 + bl;
            const int n = ntile * 16 + col;
            if (n < a.N) {
                float v = fin[bl][col] + pre_bias[0];
                if (a.act == ACT_RELU) v = fmaxf(v, 0.f);
                else if (a.act == ACT_SIGMOID) v = sigmoidf_(v);
                if (out) out[(int64_t)b * a.ldo + n] = v;
                if (a.out2) a.out2[(int64_t)b * a.ldo2 + n] = v;
                if (a.outf) a.outf[frag_idx(b, a.outf_k0 + n, a.ntf)] = v;
                if (track && !pre_done) a.hist[(int64_t)b * a.ldh + (int64_t)step * a.N + n] = v;
            }
        }
    } else if (EPI == EPI_ENC_LSTM) {
        const EncLstm& E = a.enc;
        const int e = threadIdx.x;
        if (e < Bh * 4 && enc_pos >= 0) {
            const int bl = e >> 2, u = e & 3, b = m0 + bl;
            const int unit = (ntile - dir * E.tiles_per_dir) * 4 + u;
            const float gi = fin[bl][u] + pre_bias[0];
            const float gf = fin[bl][4 + u] + pre_bias[1];
            const float gg = fin[bl][8 + u] + pre_bias[2];
            const float go = fin[bl][12 + u] + pre_bias[3];
            const float c2 = sigmoidf_(gf) * pre_cell + sigmoidf_(gi) * tanhf(gg);
            const float h = sigmoidf_(go) * tanhf(c2);
            E.c[dir * E.cstride + (int64_t)b * E.H + unit] = c2;
            E.h_next[dir * E.cstride + (int64_t)b * E.H + unit] = h;
            E.enc_out[((int64_t)b * E.Tmax + enc_pos) * (2 * E.H) + dir * E.H + unit] = h;
        }
    } else if (EPI == EPI_MEL_FUSED) {
        const MelFused& m = a.mf;
        const int nrow = m.nmel + PRE_DIM + 1;
        if (tid < Bh * 16) {
            const int bl = tid >> 4, col = tid & 15, b = m0 + bl;
            const int n = ntile * 16 + col;
            if (n < nrow - 1) {  // stop row handled below
                const float v = fin[bl][col] + pre_bias[0];
                if (n < m.nmel) {
                    // unguarded by done[]: the stop WG of this same launch may set it; rows past
                    // n_steps are garbage the host masks out (tts_decoder_run zero-fills them)
                    if (track) a.hist[(int64_t)b * a.ldh + (int64_t)step * m.nmel + n] = v;
                } else {
                    const float pv = fmaxf(v, 0.f);  // prenet layer 1 of step t+1
                    m.pre1[(int64_t)b * m.ldp + (n - m.nmel)] = pv;
                    if (m.pre1f) m.pre1f[frag_idx(b, n - m.nmel, a.ntf)] = pv;
                }
            }
        }
        if (ntile == stop_tile) {
            // stopnet + stop rule (tacotron2.py:219-224, 257-277): stop_flags[0] is always true;
            // [1] latches (tail > 0.8 and t > L); [2] = t > 2L; then 20 extra steps; the cap is
            // checked only in the `elif`, so a sentence whose flags are all set may pass it.
            __shared__ int sdone[64];
            const int col = (nrow - 1) & 15;
            const int bl = tid, b = m0 + tid;
            asm volatile("" : "+v"(sr_done), "+v"(sr_len), "+v"(sr_flag), "+v"(sr_count), "+v"(sr_tail),
                         "+v"(sr_bias));
            if (bl < Bh) {
                int nd = sr_done;
                if (!nd) {
                    const float logit = fin[bl][col] + sr_bias;
                    // teacher forcing (rule 2, Decoder.forward) returns the stopnet logits
                    const float stv = m.rule == 2 ? logit : sigmoidf_(logit);
                    if (track) m.stop_hist[(int64_t)b * m.stop_ldb + step] = stv;
                    const int L = sr_len;
                    if (m.rule == 2) {
                        // Decoder.forward (layers/tacotron2.py:227-247): no stop rule, the host runs
                        // exactly the teacher's step count
                        m.n_steps[b] = step + 1;
                    } else if (m.rule == 1) {
                        // Tacotron (layers/tacotron.py:459-469), t = step + 1 after the append:
                        // t > L/4 and (stop > 0.6 [float32 compare] or alignment[-1].item() > 0.6
                        // [double compare]); elif t > max_decoder_steps
                        const int t1 = step + 1;
                        if ((4 * t1 > L && (stv > 0.6f || (double)sr_tail > 0.6)) || t1 > m.max_steps) nd = 1;
                    } else {
                        const int f1 = sr_flag | ((sr_tail > 0.8f && step > L) ? 1 : 0);
                        m.flag1[b] = f1;
                        if (f1 && step > 2 * L) {
                            const int c = sr_count + 1;
                            m.count[b] = c;
                            if (c > 20) nd = 1;
                        } else if (step + 1 == m.max_steps) {
                            nd = 1;
                        }
                    }
                    if (nd) {
                        m.done[b] = 1;
                        m.n_steps[b] = step + 1;
                    }
                }
                sdone[bl] = nd;
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                int na = 0;
                for (int k = 0; k < Bh; ++k) na += sdone[k] ? 0 : 1;
                if (gridDim.y > 1) {
                    // row groups: each stop workgroup adds (1 << 16 | its active count) to the
                    // zeroed accumulator; the last to arrive owns the total (the counts travel in
                    // the atomic itself: no other data is handed over), publishes it and re-zeroes
                    const int old = atomicAdd(m.stop_acc, (1 << 16) + na);
                    if ((old >> 16) != (int)gridDim.y - 1) return;
                    na += old & 0xffff;
                    (void)atomicExch(m.stop_acc, 0);
                }
                *reinterpret_cast<int2*>(m.state_next) = make_int2(step + 1, na);
            }
        }
    } else if (EPI == EPI_GRU) {
        // GRU cell (torch GRUCell, ATen form): r, z gates; n = tanh(W_in x + b_in + r (W_hn h + b_hn));
        // h' = (h - n) z + n; optional residual dout = h' + res
        float* out = a.out + (a.out_par >= 0 ? (int64_t)((step + a.out_par) & 1) * a.out_pstride : 0);
        const int e = threadIdx.x;
        if (e < Bh * 4) {
            const int bl = e >> 2, u = e & 3, b = m0 + bl;
            const int unit = ntile * 4 + u;
            const float r = sigmoidf_(fin[bl][u] + pre_bias[0]);
            const float z = sigmoidf_(fin[bl][4 + u] + pre_bias[1]);
            const float n = tanhf((fin[bl][8 + u] + pre_bias[2]) + r * (fin[bl][12 + u] + pre_bias[3]));
            const float h = (pre_cell - n) * z + n;
            out[(int64_t)b * a.ldo + unit] = h;
            if (a.outf) a.outf[frag_idx(b, a.outf_k0 + unit, a.ntf)] = h;
            if (a.gru.dout) a.gru.dout[(int64_t)b * a.gru.ldd + unit] = h + pre_res;
        }
    } else {
        // LSTM cell (torch LSTMCell, gate order i, f, g, o): c' = s(f)c + s(i)tanh(g); h' = s(o)tanh(c')
        float* out = a.out + (a.out_par >= 0 ? (int64_t)((step + a.out_par) & 1) * a.out_pstride : 0);
        const int e = threadIdx.x;  // blockDim >= 256 >= B*4 for the LSTM shapes (K >= 1792)
        if (e < Bh * 4) {
            const int bl = e >> 2, u = e & 3, b = m0 + bl;
            const int unit = ntile * 4 + u;
            const float gi = fin[bl][u] + pre_bias[0];
            const float gf = fin[bl][4 + u] + pre_bias[1];
            const float gg = fin[bl][8 + u] + pre_bias[2];
            const float go = fin[bl][12 + u] + pre_bias[3];
            const float c2 = sigmoidf_(gf) * pre_cell + sigmoidf_(gi) * tanhf(gg);
            a.cell[(int64_t)b * a.ldc + unit] = c2;
            const float h = sigmoidf_(go) * tanhf(c2);
            out[(int64_t)b * a.ldo + unit] = h;
            if (a.outf) a.outf[frag_idx(b, a.outf_k0 + unit, a.ntf)] = h;
        }
    }
}

template <int MT, int EPI, int ROLE>
__global__ __launch_bounds__(1024) void sgemm_kernel(const SGemmArgs a) {
    sgemm_body<MT, EPI, ROLE, false>(a);
}

// Batched launches over fragment mirrors: 4 waves, one per SIMD, each with its own MFMA pipe and
// up to 256 VGPRs.  16 waves per CU interleave load and MFMA phases in lockstep (measured: a
// B=64 dec_lstm launch 26 us with row-major activations and 16 waves, 22.7 with mirrors and 16
// waves, 12.5 with mirrors and 4 waves; MFMA alone 10.8; tools/microbench/sgemm_b64.hip).
template <int MT, int EPI, int ROLE>
__global__ __launch_bounds__(256) void sgemm_frag_kernel(const SGemmArgs a) {
    sgemm_body<MT, EPI, ROLE, true>(a);
}

// Narrow GEMMs over fragment mirrors (one 16-row group per workgroup, <= 88 workgroups at B=64):
// most CUs are idle, so the K split over 16 waves shortens each wave's dependent load chain.
template <int EPI, int ROLE>
__global__ __launch_bounds__(1024) void sgemm_frag16_kernel(const SGemmArgs a) {
    sgemm_body<1, EPI, ROLE, true>(a);
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
    if (rowmap == ROWMAP_GRU) {
        const int col = nl & 15, gate = col >> 2, unit = (nl >> 4) * 4 + (col & 3);
        if (nl < N) {
            if (k < K1)
                v = gate < 3 ? A[(size_t)(gate * H + unit) * K1 + k] : 0.f;
            else if (gate != 2)
                v = Bm[(size_t)((gate == 3 ? 2 : gate) * H + unit) * K2 + (k - K1)];
        }
    } else if (nl < N) {
        v = k < K1 ? A[(size_t)row * K1 + k] : Bm[(size_t)row * K2 + (k - K1)];
    }
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
    if (rowmap == ROWMAP_GRU) {
        const int col = nl & 15, gate = col >> 2, unit = (nl >> 4) * 4 + (col & 3);
        if (nl < N) {
            if (gate < 2) v = a[gate * H + unit] + b[gate * H + unit];
            else if (gate == 2) v = a[2 * H + unit];
            else v = b[2 * H + unit];
        }
    } else if (nl < N) {
        v = a[row] + (b ? b[row] : 0.f);
    }
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

// Narrow GEMMs (fewer n-tiles than this) split the batch into row groups of 16, one workgroup
// per (n-tile, row group): at B = 64 the fused mel launch has 22 n-tiles, and 22 workgroups
// carrying four m-tiles each leave 234 CUs idle while they run 4x the MFMAs.  Wide GEMMs keep
// every m-tile in one workgroup, which then reads each weight fragment once for the whole batch.
// TTS_SGEMM_SPLIT overrides the n-tile threshold (0: never split).
static int split_below() {
    static const int v = [] {
        const char* e = std::getenv("TTS_SGEMM_SPLIT");
        return e && e[0] ? std::atoi(e) : 128;
    }();
    return v;
}

template <int EPI, int ROLE>
static hipError_t launch_role(const SGemmArgs& a, hipStream_t s) {
    // row-major: 16 waves (waves past K's chunk count contribute zeros); the epilogues give every
    // (row, column) of the tile its own thread, B * 16 <= 1024
    const int ntiles = (a.N + 15) / 16;
    const dim3 grid(ntiles), block(MAX_WAVES * 64);
    const int mt = (a.B + 15) / 16;
    // (the encoder LSTM, whose K = 256 steps are launch-latency bound, stays row-major: mirrors
    // of its h measured no faster)
    bool frag = a.B > 1 && a.nseg >= 1 && EPI != EPI_ENC_LSTM;
    for (int i = 0; i < a.nseg; ++i) frag = frag && a.seg[i].pf != nullptr;
    if (frag) {
        // 256 threads: the element-per-thread epilogues need B * 16 <= 256 for the linear and
        // fused-mel tiles (row groups of 16) and B * 4 <= 256 for the gate tiles
        if (a.ntf < mt) return hipErrorInvalidValue;
        const dim3 fb(256);
        if (EPI == EPI_LINEAR || EPI == EPI_MEL_FUSED || ntiles < split_below())
            hipLaunchKernelGGL((sgemm_frag16_kernel<EPI, ROLE>), dim3(ntiles, mt), block, 0, s, a);
        else if (mt <= 1)
            hipLaunchKernelGGL((sgemm_frag_kernel<1, EPI, ROLE>), grid, fb, 0, s, a);
        else if (mt <= 2)
            hipLaunchKernelGGL((sgemm_frag_kernel<2, EPI, ROLE>), grid, fb, 0, s, a);
        else
            hipLaunchKernelGGL((sgemm_frag_kernel<4, EPI, ROLE>), grid, fb, 0, s, a);
        return hipGetLastError();
    }
    if (a.B == 1)
        hipLaunchKernelGGL((sgemm_kernel<0, EPI, ROLE>), grid, block, 0, s, a);
    else if (mt <= 1)
        hipLaunchKernelGGL((sgemm_kernel<1, EPI, ROLE>), grid, block, 0, s, a);
    else if (ntiles < split_below())
        hipLaunchKernelGGL((sgemm_kernel<1, EPI, ROLE>), dim3(ntiles, mt), block, 0, s, a);
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
        case ROLE_MEL_FUSED: return launch_role<EPI_MEL_FUSED, ROLE_MEL_FUSED>(a, s);
        case ROLE_ENC_LSTM: return launch_role<EPI_ENC_LSTM, ROLE_ENC_LSTM>(a, s);
        case ROLE_T_PRENET1: return launch_role<EPI_LINEAR, ROLE_T_PRENET1>(a, s);
        case ROLE_T_PRENET2: return launch_role<EPI_LINEAR, ROLE_T_PRENET2>(a, s);
        case ROLE_T_ATT_GRU: return launch_role<EPI_GRU, ROLE_T_ATT_GRU>(a, s);
        case ROLE_T_QUERY: return launch_role<EPI_LINEAR, ROLE_T_QUERY>(a, s);
        case ROLE_T_PROJ: return launch_role<EPI_LINEAR, ROLE_T_PROJ>(a, s);
        case ROLE_T_DEC_GRU: return launch_role<EPI_GRU, ROLE_T_DEC_GRU>(a, s);
        case ROLE_T_MEL: return launch_role<EPI_LINEAR, ROLE_T_MEL>(a, s);
        case ROLE_T_PRE1_STOP: return launch_role<EPI_MEL_FUSED, ROLE_T_PRE1_STOP>(a, s);
        default: return hipErrorInvalidValue;
    }
}

// Folded weights of the fused mel/prenet-1/stop GEMM (logical row-major [nmel+257][K], fp64
// accumulation, rounded once):  rows [0,nmel) = W_mel;  [nmel, nmel+256) = W1 W_mel;
// nmel+256 = [w_s_h | 0] + w_s_mel W_mel.  Biases b_mel, W1 b_mel (+ b1: the BatchNorm prenet's
// folded shift), b_s + w_s_mel b_mel.
__global__ void fold_mel_kernel(const float* Wm, const float* bm, const float* W1, const float* b1, const float* ws,
                                const float* bs, int nmel, int K, int hdec, float* Wf, float* bf) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int nrow = nmel + PRE_DIM + 1;
    if (i >= (int64_t)nrow * (K + 1)) return;
    const int n = i / (K + 1), k = i % (K + 1);  // k == K: bias
    double v = 0.0;
    if (n < nmel) {
        v = k < K ? Wm[(int64_t)n * K + k] : bm[n];
    } else if (n < nmel + PRE_DIM) {
        const float* w1 = W1 + (int64_t)(n - nmel) * nmel;
        for (int m = 0; m < nmel; ++m) v += (double)w1[m] * (k < K ? Wm[(int64_t)m * K + k] : bm[m]);
        if (k == K && b1) v += b1[n - nmel];
    } else {
        v = k < K ? (k < hdec ? ws[k] : 0.0) : bs[0];
        for (int m = 0; m < nmel; ++m) v += (double)ws[hdec + m] * (k < K ? Wm[(int64_t)m * K + k] : bm[m]);
    }
    if (k < K)
        Wf[(int64_t)n * K + k] = (float)v;
    else
        bf[n] = (float)v;
}

hipError_t fold_mel_weights(const float* Wm, const float* bm, const float* W1, const float* b1, const float* ws,
                            const float* bs, int nmel, int K, int hdec, float* Wf, float* bf, hipStream_t s) {
    const int64_t total = (int64_t)(nmel + PRE_DIM + 1) * (K + 1);
    hipLaunchKernelGGL(fold_mel_kernel, dim3((total + 255) / 256), dim3(256), 0, s, Wm, bm, W1, b1, ws, bs, nmel, K,
                       hdec, Wf, bf);
    return hipGetLastError();
}

__global__ void fold_linear_bn_kernel(const float* W, const float* b, const float* gamma, const float* beta,
                                      const float* mean, const float* var, int rows, int cols, float eps, float* Wout,
                                      float* bout) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)rows * (cols + 1)) return;
    const int n = i / (cols + 1), k = i % (cols + 1);  // k == cols: bias
    const double sc = (double)gamma[n] / sqrt((double)var[n] + (double)eps);
    if (k < cols)
        Wout[(int64_t)n * cols + k] = (float)(sc * W[(int64_t)n * cols + k]);
    else
        bout[n] = (float)(sc * ((b ? (double)b[n] : 0.0) - mean[n]) + beta[n]);
}

hipError_t fold_linear_bn(const float* W, const float* b, const float* gamma, const float* beta, const float* mean,
                          const float* var, int rows, int cols, float eps, float* Wout, float* bout, hipStream_t s) {
    const int64_t total = (int64_t)rows * (cols + 1);
    hipLaunchKernelGGL(fold_linear_bn_kernel, dim3((total + 255) / 256), dim3(256), 0, s, W, b, gamma, beta, mean, var,
                       rows, cols, eps, Wout, bout);
    return hipGetLastError();
}

}  // namespace tts

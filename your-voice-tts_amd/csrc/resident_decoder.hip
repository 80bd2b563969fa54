// Resident batch-1 decoder: one persistent launch for the whole decoder loop (see resident.h).
//
// Per step t on compute unit c (512 threads = 8 waves; thread (r = tid/32, ks = tid%32) owns
// gate row r = g*4 + u of units 4c..4c+3 and the k-slice {i*128 + 4ks .. +4}):
//   1. attention-LSTM partial over [ctx_{t-1} | h_att_{t-1}]            (all waves, VGPR weights)
//   2. wave 0: wait pre1_t (+ continue flag), prenet-2 row c, publish; gather the 256 rows
//   3. prenet part, row sums, LSTM cell of units 4c..4c+3, publish h_att_t   (tacotron2.py:195-197)
//   4. gather h_att_t; 5. CUs < 128: query row c, publish                     (common_layers.py:179)
//   6. decoder-LSTM partial over [h_att_t | h_dec_{t-1}]                  (LDS weights)
//   7. CU 255: energies, sigmoid, forward attention + mask, context, publish ctx_t and the tail
//      (common_layers.py:178-182, 199-223, 239-253)
//   8. gather ctx_t; 9. context part, cell, publish h_dec_t               (tacotron2.py:206-208)
//  10. gather h_dec_t (the prenet-1 row weights of step 11 in flight from the XCD's L2);
//  11. every wave: one folded prenet-1 row of this XCD's copy -> XCD-local publish; the XCD's
//      stop CU (rank 0), wave 3: the stop row -> sigmoid + stop rule -> XCD-local continue flag
//      (tacotron2.py:214-224, 256-277).  Mel row c of step t is written by wave 4 during step
//      t+1's h_att gather (after the loop for the last step).
// Reductions keep fixed orders (bitwise run-to-run deterministic).
#include "handoff.h"
#include "resident.h"

namespace tts {
namespace {
using namespace handoff;

// LSTM cell of units 4c..4c+3 from the 16 gate sums (row g*4 + u, torch order i, f, g, o): lanes
// 0..15 evaluate one gate nonlinearity each in parallel; lanes 0..3 pull f, g, o from lanes u+4,
// u+8, u+12 by DPP row shifts and update (c, h) as the sgemm LSTM epilogue does (its nonlinearities
// by the hardware-exp2 forms sigmoid_cell / tanh_cell, common.h).
// Call with lanes 0..15 of wave 0 active; returns h in lanes 0..3 and updates c there.
__device__ __forceinline__ float lstm_cell16(float pre, float& c) {
    const int k = threadIdx.x;
    const float act = (k >> 2) == 2 ? tanh_cell(pre) : sigmoid_cell(pre);
    const float f = dpp_move<0x104, 0xf>(act, 0.f);   // row_shl:4
    const float g = dpp_move<0x108, 0xf>(act, 0.f);   // row_shl:8
    const float o = dpp_move<0x10C, 0xf>(act, 0.f);   // row_shl:12
    const float c2 = f * c + act * g;
    c = c2;
    return o * tanh_cell(c2);
}
// sigmoid from the hardware exp2 / reciprocal for the attention energies (sigmoid_cell's form)
__device__ __forceinline__ float sigmoid_fast(float x) {
    return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-x * 1.4426950408889634f));
}

__device__ __forceinline__ float dot4(float4 w, float4 x, float acc) {
    acc = fmaf(w.x, x.x, acc);
    acc = fmaf(w.y, x.y, acc);
    acc = fmaf(w.z, x.z, acc);
    return fmaf(w.w, x.w, acc);
}
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
// Sums over each half-wave (lanes 0-31, 32-63) by DPP row scans: the totals land in lanes 31
// and 63 (other lanes hold partial scans).  No LDS round trip per level.
__device__ __forceinline__ float sum32_dpp(float v) {
    v += dpp_move<0x111, 0xf>(v, 0.f);  // row_shr:1
    v += dpp_move<0x112, 0xf>(v, 0.f);  // row_shr:2
    v += dpp_move<0x114, 0xf>(v, 0.f);  // row_shr:4
    v += dpp_move<0x118, 0xf>(v, 0.f);  // row_shr:8
    v += dpp_move<0x142, 0xa>(v, 0.f);  // row_bcast:15 into rows 1, 3
    return v;
}

// Candidate slot s (0..15) of the attention fast path: the window W(n) = {(n-2) mod L} +
// [n-1, min(n+2, L-1)] (slots 0-4), then p and p + 1 for every p of the previous window W(n')
// (slots 5-14); -1 = unused.  Duplicates are allowed (same value written twice).
__device__ __forceinline__ int res_window(int k, int nn, int L) {
    if (k == 0) return nn >= 2 ? nn - 2 : nn - 2 + L;
    const int clo = nn >= 1 ? nn - 1 : L - 1, chi = min(nn + 2, L - 1);
    const int p = clo + k - 1;
    return p <= chi ? p : -1;
}
__device__ __forceinline__ int res_candidate(int s, int nn, int np, int L) {
    if (s < 5) return res_window(s, nn, L);
    if (s >= 15) return -1;
    const int p = res_window((s - 5) >> 1, np, L);
    if (p < 0) return -1;
    const int q = p + ((s - 5) & 1);
    return q < L ? q : -1;
}

constexpr int SM_WDL = 16 * 16 * 32 * 4;  // floats of the decoder-LSTM LDS weight image (128 KiB)
constexpr int SM_ST = 64;                  // biases, cell states, stop-rule state
constexpr int SM_RQ = 4 * 64 * 4;          // query row [4 i4][64 lanes] float4 | attention CU scratch
constexpr int SM_RM = 2 * 6 * 64 * 4 + 2 * 256;  // mel row c, stop row: [2][6][64] float4 | row c + energy partials
constexpr int SM_PROF = 2 * 16;            // RES_PHASES tick accumulators (long long)
constexpr int SM_FLOATS = SM_WDL + HATT + HDEC + (ENC + 16) + PRE + ADIM + 16 + 16 + SM_ST + SM_RQ + SM_RM + SM_PROF + PRE;
static_assert(SM_RM >= 6 * 64 * 4 + RES_WAVES * RES_LMAX, "attention CU partials");
static_assert(SM_RQ >= 3 * RES_LMAX + 2 * RES_WAVES + 16 + ADIM, "attention CU scratch");
static_assert(SM_RQ >= 2 * (RES_LMAX + 32) + RES_LMAX + RES_WAVES, "general attention form: weights, energies");
static_assert(SM_RM >= 2 * 6 * 64 * 4 + RES_LMAX + 32, "general attention form: cumulative weights");
static_assert(RES_LMAX == 4 * 64 && RES_LMAX == 32 * RES_WAVES, "4 positions per lane, one per wave of 32 CUs");

// PROF: the profiling re-run's instantiation (phase marks, event trace); the production kernel
// compiles every measurement site out (their pointers, ticks and step compares otherwise stay live
// across the step loop in scalar registers, which this kernel already spills)
// GEN: the general attention form (resident.h): the attention of each XCD spread over its CUs
template <bool PROF, bool GEN>
__global__ __launch_bounds__(RES_THREADS, 1) void resident_decoder_kernel(const ResArgs a) {
    const int c = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = tid >> 5, ks = tid & 31;
    extern __shared__ __align__(16) float sm[];
    float4* wdl = reinterpret_cast<float4*>(sm);  // [16 i4][16 r][32 ks]
    float* xh_att = sm + SM_WDL;
    float* xh_dec = xh_att + HATT;
    float* xctx = xh_dec + HDEC;  // [ENC] context, [ENC] = stop-rule tail
    float* xpre = xctx + ENC + 16;
    float* xq = xpre + PRE;
    float* gates = xq + ADIM;  // [16]
    int* flags = reinterpret_cast<int*>(gates + 16);  // [0] stop seen, [1] abort
    float* st = gates + 32;    // [0,16) b_att, [16,32) b_dec (row g*4+u), [32,36) c_att, [36,40) c_dec,
                               // [40,44) h_att, [44,48) h_dec of units 4c+u, [48] mel bias, [49] stop
                               // bias, [50] flag1, [51] count (int bits, stop lane)
    float* rq = st + SM_ST;    // query row (CUs < 128) | attention CU: aold, an, scr, v
    float* rm = rq + SM_RQ;    // mel row c, stop row (stop CU) | attention CU: row c + energy partials
    float* abuf = rq;                 // [2][RES_LMAX] previous alpha, ping-pong by step parity
    float* an = abuf + 2 * RES_LMAX;  // unnormalised forward weights of this step
    float* scr = an + RES_LMAX;       // [2 * RES_WAVES] + candidate values [16]
    float* xv = scr + 2 * RES_WAVES + 16;
    float* red = rm + 6 * 64 * 4;  // [RES_WAVES][RES_LMAX]
    long long* pacc = reinterpret_cast<long long*>(rm + SM_RM);
    float* xp1 = rm + SM_RM + SM_PROF;  // pre1_t (prenet layer 1 output) gathered by wave 0
    // general attention form (every CU): attention weights of the last two steps, zero-padded by
    // 16 on both sides for the location convolution ([2][GW_PAD], position j at j + 16), the
    // gathered energies, the transition agent's wave partials; the cumulative weights (padded)
    // in the tail of rm (the mask form's attention-CU partials; no mel or stop row there)
    constexpr int GW_PAD = RES_LMAX + 32;
    float* gw = rq;                     // [2][GW_PAD]
    float* geg = rq + 2 * GW_PAD;       // [RES_LMAX]
    float* gts = geg + RES_LMAX;        // [RES_WAVES]
    float* gcum = rm + 2 * 6 * 64 * 4;  // [GW_PAD]
    // optional phase timing (thread 0 of CU 0 and of the logging attention CU)
    bool prof = false;
    long long plast = 0;
    // event trace of the profiling re-run (RES_TRACE_STEPS steps x RES_TRACE_EV events per CU,
    // wall_clock64 ticks): measurement only
    long long* trace = PROF && a.prof ? a.prof + 2 * RES_PHASES + (size_t)c * RES_TRACE_STEPS * RES_TRACE_EV : nullptr;
#define RES_EV(t, k)                                                                                \
    if (PROF && trace && (t) < RES_TRACE_STEPS) trace[(t) * RES_TRACE_EV + (k)] = (long long)wall_clock64();
#define RES_MARK(k)                                     \
    if (PROF && prof && tid == 0) {                     \
        const long long now = (long long)wall_clock64(); \
        pacc[k] += now - plast;                         \
        plast = now;                                    \
    }

    // ---- weights (loaded once per call) and initial state
    float4 wa[14], wdc[4];
    constexpr int KF = HDEC + ENC;  // folded-row length
    {
        const float4* p = a.w.wa + (size_t)c * 14 * RES_THREADS + tid;
#pragma unroll
        for (int i = 0; i < 14; ++i) wa[i] = p[(size_t)i * RES_THREADS];
        const float4* q = a.w.wdc + (size_t)c * 4 * RES_THREADS + tid;
#pragma unroll
        for (int i = 0; i < 4; ++i) wdc[i] = q[(size_t)i * RES_THREADS];
        if (wave == 2 && c < a.nmel)  // mel row c in LDS
            for (int i = 0; i < 6; ++i) reinterpret_cast<float4*>(rm)[i * 64 + lane] = ld4(a.w.wf + (size_t)c * KF + i * 256 + lane * 4);
        const float4* l = a.w.wdl + (size_t)c * (SM_WDL / 4);
        for (int i = tid; i < SM_WDL / 4; i += RES_THREADS) wdl[i] = l[i];
    }
    if (tid < 16) {
        st[tid] = a.w.ba[c * 16 + tid];
        st[16 + tid] = a.w.bd[c * 16 + tid];
    }
    if (tid < 4) {
        st[32 + tid] = a.c_att[4 * c + tid];
        st[36 + tid] = a.c_dec[4 * c + tid];
    }
    if (tid == 0) st[48] = c < a.nmel ? a.w.bf[c] : 0.f;
    if (tid == 1) st[49] = a.w.bf[a.nmel + PRE];
    for (int k = tid; k < HATT; k += RES_THREADS) {
        xh_att[k] = a.h_att[a.hps + k];  // step 0 reads slot 1 (decoder_init_kernel)
        xh_dec[k] = a.h_dec[a.hps + k];
    }
    for (int k = tid; k < ENC; k += RES_THREADS) xctx[k] = a.xa[PRE + k];
    if (tid == 0) {
        flags[0] = 0;
        flags[1] = 0;
        for (int k = 0; k < RES_PHASES; ++k) pacc[k] = 0;
    }
    __syncthreads();
    const long long tmo = a.timeout_ticks;
    // ---- XCD discovery: prenet-2 is computed and exchanged inside each XCD (same-L2 hand-off).
    // Every CU publishes its XCC id; each reads the table, takes rank = #CUs of its XCD before it,
    // and computes rows [rank * 256 / n, (rank + 1) * 256 / n) of its XCD's copy of prenet-2.
    int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7;
    const unsigned setup_tag = (a.salt << 14) | 0x3FFFu;
    if (tid == 0) publish(a.gran + GR_SETUP + c, setup_tag, __int_as_float(xcc));
    if (wave == 0) {
        float v4[4];
        const bool ok = sweep<4>(a.gran, setup_tag, v4, [&](int i) { return GR_SETUP + lane * 4 + i; }, tmo);
        int rank = 0, nx = 0, nmin = RES_CUS, nmax = 0;
        const int xref = __builtin_amdgcn_readfirstlane(__float_as_int(v4[0]) & 7);  // XCD of CU 0
        for (int k = 0; k < 8; ++k) {
            int cnt = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int x = __float_as_int(v4[i]) & 7;
                cnt += __popcll(__ballot(x == k));
                if (k == xcc) rank += __popcll(__ballot(x == k && lane * 4 + i < c));
            }
            if (k == xcc) nx = cnt;
            if (cnt > 0) nmin = min(nmin, cnt);
            nmax = max(nmax, cnt);
        }
        // (general form: CU rank k owns context channels [16 k, 16 k + 16) of its XCD's copy)
        if (GEN && nmax > RES_MIN_CUS_PER_XCD) nmin = 0;
        if (lane == 0) {
            int* fl = reinterpret_cast<int*>(flags);
            fl[2] = rank;
            fl[3] = nx;
            fl[4] = xref;
            if (!ok) { flags[1] = 1; fail(a.status, 6); }
            else if (nmin < RES_MIN_CUS_PER_XCD) { flags[1] = 1; fail(a.status, RES_STATUS_PLACEMENT); }
        }
    }
    __syncthreads();
    if (flags[1]) return;
    const int rank = flags[2], nx = flags[3];
    const int p2lo = rank * PRE / nx, p2hi = (rank + 1) * PRE / nx;
    // this wave's prenet-2 row and prenet-1 row of the XCD's copies (nx >= 32: at most one per wave)
    const int r0 = p2lo + wave;
    const bool has_row = r0 < p2hi;
    const float4 wp0 = has_row ? ld4(a.w.w2 + r0 * PRE + lane * 4) : float4{0.f, 0.f, 0.f, 0.f};
    const float bp1 = has_row ? a.w.bf[a.nmel + r0] : 0.f;
    const float bp2 = has_row ? a.w.b2[r0] : 0.f;
    // folded prenet-1 row (re-read from the XCD's L2 every step: no register or LDS room); a wave
    // without a row loads row 0 and discards it (no branch around the loads)
    const float* w1p = a.w.wf + (size_t)(a.nmel + (has_row ? r0 : 0)) * KF + lane * 4;
    const bool stop_cu = rank == 0;  // this XCD's stopnet + stop rule
    if (stop_cu && wave == 3)
        for (int i = 0; i < 6; ++i)
            reinterpret_cast<float4*>(rm)[(6 + i) * 64 + lane] = ld4(a.w.wf + (size_t)(a.nmel + PRE) * KF + i * 256 + lane * 4);
    // query rows 4 rank .. 4 rank + 3 of this XCD's copy: wave w holds half (w & 1) of row 4 rank + w / 2
    const int qrow = 4 * rank + (wave >> 1), qhalf = wave & 1;
    const float4 wq0 = ld4(a.w.wq + qrow * HATT + qhalf * 512 + lane * 4);
    const float4 wq1 = ld4(a.w.wq + qrow * HATT + qhalf * 512 + 256 + lane * 4);
    const int L = a.L;
    const bool att_cu = !GEN && rank == nx - 1;       // the last CU of each XCD runs its attention copy
    const bool xlog = xcc == flags[4];                // the XCD whose copies write the outputs
    const bool att_log = att_cu && xlog;              // ... alignment rows
    prof = PROF && a.prof != nullptr && a.prof_marks && (c == 0 || att_log);
    if (prof && tid == 0) plast = (long long)wall_clock64();
    int n = 0, n_prev = 0;
    float ufa = 0.f, vb = 0.f, ex = 0.f, erow[4] = {0.f, 0.f, 0.f, 0.f}, ptc[4] = {0.f, 0.f, 0.f, 0.f};
    // (volatile buffer loads: the compiler may not sink them past the volatile polls of the h_att
    // gather to their use in the context, where their latency would sit on the critical path)
    const auto renc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.enc), (short)0, L * ENC * 4, 0x00020000);
    const auto rpt = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.Pt), (short)0, ADIM * a.Lcap * 4, 0x00020000);
    auto prefetch_rows = [&](int nn) {
        // the rows the context can use after the mask: (nn-2) mod L and [nn-1, nn+2]
        const int cx = (nn - 2 + L) % L, clo = nn >= 1 ? nn - 1 : L - 1, chi = min(nn + 2, L - 1);
        ex = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(renc, (cx * ENC + tid) * 4, 0, VOLATILE_AUX));
#pragma unroll
        for (int k = 0; k < 4; ++k)
            erow[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                renc, clo + k <= chi ? ((clo + k) * ENC + tid) * 4 : OOB_OFF, 0, VOLATILE_AUX));
    };
    if (att_cu) {
        n = a.nidx[0];
        ufa = a.u[0];
        vb = a.v_b[0];
        for (int j = tid; j < L; j += RES_THREADS) abuf[j] = a.alpha[j];  // step 0 reads buffer 0
        if (tid < ADIM) xv[tid] = a.v[tid];
        prefetch_rows(n);
    }
    // ---- general attention form: this CU's slices (position rank + 32 wave; context channels
    // 16 rank + 2 wave + {0, 1} at this lane's positions gpos(i) = (i >> 1) 128 + 2 lane + (i & 1))
    // and the attention state, replicated in every wave of every CU
    const int gf = GEN ? a.gen : 0;
    const int s_e = GR_EX + xcc * RES_LMAX;  // this XCD's energy slots
    float gu = 0.5f, gtb = 0.f;              // forward attention u, transition agent bias
    int gwin = -1, gn = 1;                   // windowing index, the mask's argmax n
    float gv0 = 0.f, gv1 = 0.f, gp0 = 0.f, gp1 = 0.f, gl0 = 0.f, gl1 = 0.f;  // v, P, location term: dims lane, lane + 64
    float gtw[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) gtw[k] = 0.f;
    // location_conv (2 -> 32 filters, k 31, pad 15) at position rank + 32 wave over [weights;
    // cumulative weights] (padded LDS rows), then location_dense (32 -> 128) for dims lane and
    // lane + 64 (common_layers.py:86-104, 166-171): lane (f = lane & 31, channel lane >> 5) sums
    // its 31 taps, the two channels meet by a lane swap, every lane reads the 32 filter outputs
    auto gen_location = [&](const float* wrow) {
        const int pe = rank + 32 * wave;
        if (pe >= L) return;
        const float* src = (lane < 32 ? wrow : gcum) + pe + 1;  // cat[c][pe + k - 15] = src[k]
        const float4* wc = reinterpret_cast<const float4*>(a.loc_conv) + lane * 8;
        float sacc = 0.f;
#pragma unroll
        for (int q = 0; q < 8; q += 2) {
            const float4 w0 = wc[q], w1_ = wc[q + 1];
            sacc = fmaf(w0.x, src[4 * q], sacc);
            sacc = fmaf(w0.y, src[4 * q + 1], sacc);
            sacc = fmaf(w0.z, src[4 * q + 2], sacc);
            sacc = fmaf(w0.w, src[4 * q + 3], sacc);
            sacc = fmaf(w1_.x, src[4 * q + 4], sacc);
            sacc = fmaf(w1_.y, src[4 * q + 5], sacc);
            sacc = fmaf(w1_.z, src[4 * q + 6], sacc);
            sacc = fmaf(w1_.w, src[4 * q + 7], sacc);
            asm volatile("" ::: "memory");  // two weight loads in flight at a time (registers)
        }
        const float tot = sacc + __shfl_xor(sacc, 32, 64);  // lane f < 32: filter f
        const float4* wd0 = reinterpret_cast<const float4*>(a.loc_dense + lane * NLOC);
        const float4* wd1 = reinterpret_cast<const float4*>(a.loc_dense + (lane + 64) * NLOC);
        float l0 = 0.f, l1 = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const float4 u0 = wd0[q], u1 = wd1[q];
            const float f0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tot), 4 * q));
            const float f1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tot), 4 * q + 1));
            const float f2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tot), 4 * q + 2));
            const float f3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tot), 4 * q + 3));
            l0 = fmaf(u0.x, f0, l0); l0 = fmaf(u0.y, f1, l0); l0 = fmaf(u0.z, f2, l0); l0 = fmaf(u0.w, f3, l0);
            l1 = fmaf(u1.x, f0, l1); l1 = fmaf(u1.y, f1, l1); l1 = fmaf(u1.z, f2, l1); l1 = fmaf(u1.w, f3, l1);
            asm volatile("" ::: "memory");
        }
        gl0 = l0;
        gl1 = l1;
    };
    if constexpr (GEN) {
        vb = a.v_b[0];
        gu = a.u[0];
        gn = a.nidx[0];
        if (gf & GEN_WINDOW) gwin = a.win0[0];
        if (gf & GEN_TA) {
            gtb = a.ta_b[0];
#pragma unroll
            for (int k = 0; k < 3; ++k) gtw[k] = a.ta_w[3 * tid + k];
        }
        gv0 = a.v[lane];
        gv1 = a.v[lane + 64];
        const int pe = rank + 32 * wave;
        if (pe < L) {
            gp0 = a.Pt[(int64_t)lane * a.Lcap + pe];
            gp1 = a.Pt[(int64_t)(lane + 64) * a.Lcap + pe];
        }
        // padded rows: [0] the previous alpha (forward attention; read at step 0), [1] the initial
        // attention_weights (the location input of step 0; step 0 then overwrites it)
        for (int k = tid; k < GW_PAD; k += RES_THREADS) {
            const int j = k - 16;
            const bool ok = j >= 0 && j < L;
            gw[k] = ok ? a.alpha[j] : 0.f;
            gw[GW_PAD + k] = ok && (gf & GEN_LOCATION) ? a.att_w0[j] : 0.f;
            gcum[k] = ok && (gf & GEN_LOCATION) ? a.att_cum0[j] : 0.f;
        }
        __syncthreads();
        if (gf & GEN_LOCATION) gen_location(gw + GW_PAD);
    }
    const bool stop_lane = stop_cu && wave == 3 && lane == 0;
    if (stop_lane) {
        reinterpret_cast<int*>(st)[50] = a.flag1[0];
        reinterpret_cast<int*>(st)[51] = a.count[0];
    }
    u64* Gx = a.gran + GR_PRE2X + xcc * PRE;  // this XCD's prenet-2 slots (parity offset added below)
    u64* Gq = a.gran + GR_QX + xcc * 2 * ADIM;   // this XCD's query half-rows
    u64* Gc = a.gran + GR_CTXX + xcc * GR_CTXX_STRIDE;  // this XCD's context + tail
    u64* G1 = a.gran + GR_P1X + xcc * GR_P1X_STRIDE;    // this XCD's prenet-1 rows + continue flag
    // the gathers' pair loads: one buffer resource over both parities' granules, slot offsets
    const auto rg = __builtin_amdgcn_make_buffer_rsrc(a.gran, (short)0, 2 * GR_TOTAL * 8, 0x00020000);
    const int s_x = GR_PRE2X + xcc * PRE, s_q = GR_QX + xcc * 2 * ADIM, s_c = GR_CTXX + xcc * GR_CTXX_STRIDE,
              s_1 = GR_P1X + xcc * GR_P1X_STRIDE;
    const int pk = wave * 64 + lane;  // this lane's pair of a gather over all waves
    // mel row c of step tt from xh_dec / xctx (= h_dec_tt, ctx_tt), by one wave
    auto mel_row = [&](int tt) {
        if (c >= a.nmel) return;
        const float4* wm = reinterpret_cast<const float4*>(rm) + lane;
        float sm_ = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) sm_ = dot4(wm[i * 64], ld4(xh_dec + i * 256 + lane * 4), sm_);
#pragma unroll
        for (int i = 4; i < 6; ++i) sm_ = dot4(wm[i * 64], ld4(xctx + (i - 4) * 256 + lane * 4), sm_);
        sm_ = wave_sum_dpp(sm_);
        if (lane == 0 && tt < a.hist_cap) a.mel_hist[(int64_t)tt * a.nmel + c] = sm_ + st[48];
    };
    int t = 0;
    for (;; ++t) {
        u64* G = a.gran + (t & 1) * GR_TOTAL;          // this step's granules
        // tags E+1 .. E+7 (never 0): the step count wraps at 2048 inside its 11 bits (a granule
        // slot is rewritten every second step, so only step t-2's tag can be stale there; runs
        // reach the Synthesizer's 3000-step cap, server/synthesizer.py:66), the previous step's
        // prenet-1 tag EP6 computed on its own wrapped count
        const unsigned E = (a.salt << 14) | (((unsigned)t & 2047u) << 3);
        const unsigned EP6 = ((a.salt << 14) | (((unsigned)(t - 1) & 2047u) << 3)) + 6u;
        // 1) attention LSTM over [ctx_{t-1} | h_att_{t-1}]
        // (two accumulators each: dependency chains of 24 and 16 FMAs instead of 48 and 32, ahead
        // of the pre1 poll)
        float aa[2] = {0.f, 0.f};
#pragma unroll
        for (int i = 2; i < 6; ++i) aa[i & 1] = dot4(wa[i], ld4(xctx + (i - 2) * 128 + ks * 4), aa[i & 1]);
#pragma unroll
        for (int i = 6; i < 10; ++i) aa[i & 1] = dot4(wa[i], ld4(xh_att + (i - 6) * 128 + ks * 4), aa[i & 1]);
        asm volatile("" ::: "memory");  // bound the hoisted LDS loads (register pressure)
#pragma unroll
        for (int i = 10; i < 14; ++i) aa[i & 1] = dot4(wa[i], ld4(xh_att + (i - 6) * 128 + ks * 4), aa[i & 1]);
        float acc_a = aa[0] + aa[1];
        // decoder LSTM over h_dec_{t-1}, also while pre1 is in flight
        float ad[2] = {0.f, 0.f};
#pragma unroll 2
        for (int i = 8; i < 16; ++i)
            ad[i & 1] = dot4(wdl[(i * 16 + r) * 32 + ks], ld4(xh_dec + (i - 8) * 128 + ks * 4), ad[i & 1]);
        float acc_d = ad[0] + ad[1];
        // 2) prenet layer 2: wave 0 gathers this XCD's pre1_t (+ the previous step's continue flag);
        //    every wave computes its row of this XCD's copy, publishes it XCD-locally; wave 0 gathers
        // (waves 0, 1: the 256 rows as pairs; wave 2, lane 0: the flag)
        if (wave < 3) {
            const int gp = s_1 + ((t & 1) ^ 1) * GR_TOTAL;
            bool ok = true;
            if (t == 0) {
                if (wave == 0) {
                    const float4 v = ld4(a.pre1 + lane * 4);  // go frame's layer 1 (enqueue_prenet_go)
                    xp1[lane * 4] = v.x; xp1[lane * 4 + 1] = v.y; xp1[lane * 4 + 2] = v.z; xp1[lane * 4 + 3] = v.w;
                }
            } else {
                float p0 = 0.f, p1 = 0.f;
                for (int i = 0; i < a.sleep_p1; ++i) __builtin_amdgcn_s_sleep(4);
                if (wave < 2) {
                    ok = sweep_pair(rg, gp + 2 * pk, true, EP6, p0, p1, tmo);
                    xp1[2 * pk] = p0;
                    xp1[2 * pk + 1] = p1;
                } else {
                    ok = sweep_pair(rg, lane == 0 ? gp + PRE : -1, false, EP6, p0, p1, tmo);
                    if (lane == 0 && ok && p0 == 0.f) flags[0] = 1;
                }
            }
            RES_MARK(0);
            if (lane == 0 && !ok) { flags[1] = 1; fail(a.status, 1, t); }
        }
        __syncthreads();  // P1
        if (tid == 0) { RES_EV(t, 0) }
        if (flags[0] | flags[1]) break;
        {
            const float4 x = ld4(xp1 + lane * 4);
            u64* gx = Gx + (t & 1) * GR_TOTAL;
            if (has_row) {
                const float s0 = wave_sum_dpp(dot4(wp0, x, 0.f));
                if (lane == 0) publish_xcd(gx + r0, E + 1, fmaxf(s0 + bp2, 0.f));
            }
            RES_MARK(1);
            if (wave < 2) {
                for (int i = 0; i < a.sleep_pre2; ++i) __builtin_amdgcn_s_sleep(4);
                float q0, q1;
                const bool ok = sweep_pair(rg, s_x + (t & 1) * GR_TOTAL + 2 * pk, true, E + 1, q0, q1, tmo);
                xpre[2 * pk] = q0;
                xpre[2 * pk + 1] = q1;
                if (!ok && lane == 0) { flags[1] = 1; fail(a.status, 7, t); }
            }
        }
        __syncthreads();  // B1
        if (tid == 0) { RES_EV(t, 1) }
        if (flags[1]) break;
        RES_MARK(2);
        // 3) prenet part, cell
#pragma unroll
        for (int i = 0; i < 2; ++i) acc_a = dot4(wa[i], ld4(xpre + i * 128 + ks * 4), acc_a);
        acc_a = sum32_dpp(acc_a);
        if (ks == 31) gates[r] = acc_a;
        __syncthreads();  // B2
        RES_MARK(3);
        if (tid < 16) {
            float cs = st[32 + (tid & 3)];
            const float h = lstm_cell16(gates[tid] + st[tid], cs);
            if (tid < 4) {
                st[32 + tid] = cs;
                st[40 + tid] = h;
                publish(G + GR_HATT + 4 * c + tid, E + 2, h);
                if (tid == 0) { RES_EV(t, 2) }
            }
        }
        // 4) gather h_att_t (all waves); first wave 4 writes the mel row c of step t-1 (xh_dec, xctx
        //    still hold h_dec_{t-1}, ctx_{t-1}): off the critical path of step t-1's pre1 rows.  The
        //    attention CU first issues this step's attention operands (the encoder rows the mask can
        //    keep, P at the candidate positions): in flight while h_att is awaited (a load issued
        //    before the pre1 poll instead held that poll up by its latency, vmcnt being in order, and
        //    with it the XCD's prenet-2 rows: 1.2 us per step, round-4 trace)
        if (att_cu && t > 0) {
            prefetch_rows(n);
            const int pos = res_candidate(tid >> 5, n, n_prev, L);
#pragma unroll
            for (int m = 0; m < 4; ++m)
                ptc[m] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                    rpt, pos >= 0 ? (((tid & 31) + 32 * m) * a.Lcap + pos) * 4 : OOB_OFF, 0, VOLATILE_AUX));
        }
        {
            if (wave == 4 && t > 0) mel_row(t - 1);
            for (int i = 0; i < a.sleep_hatt; ++i) __builtin_amdgcn_s_sleep(4);
            float h0, h1;
            const bool ok = sweep_pair(rg, (t & 1) * GR_TOTAL + GR_HATT + 2 * pk, true, E + 2, h0, h1, tmo);
            xh_att[2 * pk] = h0;
            xh_att[2 * pk + 1] = h1;
            if (!ok && lane == 0) { flags[1] = 1; fail(a.status, 2, t); }
        }
        __syncthreads();  // B3
        if (tid == 0) { RES_EV(t, 3) }
        if (flags[1]) break;
        RES_MARK(4);
        // 5) query half-rows of this XCD's copy (common_layers.py:179), published XCD-locally
        {
            float s = dot4(wq0, ld4(xh_att + qhalf * 512 + lane * 4), 0.f);
            s = dot4(wq1, ld4(xh_att + qhalf * 512 + 256 + lane * 4), s);
            s = wave_sum_dpp(s);
            if (lane == 0) publish_xcd(Gq + (t & 1) * GR_TOTAL + 2 * qrow + qhalf, E + 3, s);
            if (tid == 0) { RES_EV(t, 8) }
        }
        // 6) decoder LSTM over h_att_t (its h_dec_{t-1} half ran at the loop top); the attention
        //    CU does this after its attention step, which is on the critical path (there it runs
        //    while the other CUs' context gather waits out the XCD-local edge)
        if (!att_cu) {
#pragma unroll 2
            for (int i = 0; i < 8; ++i) acc_d = dot4(wdl[(i * 16 + r) * 32 + ks], ld4(xh_att + i * 128 + ks * 4), acc_d);
        }
        RES_MARK(5);
        float wdef = 0.f;  // attention CU: this thread's weight of the step (stored after h_dec is published)
        // 7) attention step.  After the forward mask the previous alpha is nonzero only on the
        //    previous window S' = W(n') = {(n'-2) mod L} + [n'-1, n'+2], so every position outside
        //    C = W(n) + S' + (S'+1) has mix = 1e-8 exactly and anj = 1e-8 * sigmoid <= 1e-8: the
        //    outputs (window weights, max(alpha), the window sum) need the energies of C only
        //    (<= 15 positions, duplicates harmless) whenever max over C >= 1e-8.  Step 0 (alpha
        //    initialised nonzero everywhere) and that rare case evaluate every position.
        if constexpr (GEN) {
            // 7') general attention form (resident.h).  This lane's encoder values of the context
            // (channels 16 rank + 2 wave + {0, 1} at its positions; volatile: issued here, in flight
            // across the query and energy hand-offs), then the query of this XCD's copy (waves 0-1)
            float2 gen_e[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int ps = (i >> 1) * 128 + 2 * lane + (i & 1);
                gen_e[i] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(
                    renc, ps < L ? (ps * ENC + 16 * rank + 2 * wave) * 4 : OOB_OFF, 0, VOLATILE_AUX));
            }
            if (wave < 2) {
                for (int i = 0; i < a.sleep_q; ++i) __builtin_amdgcn_s_sleep(1);
                float q0, q1;
                const bool ok = sweep_pair(rg, s_q + (t & 1) * GR_TOTAL + 2 * pk, true, E + 3, q0, q1, tmo);
                xq[pk] = q0 + q1;
                if (!ok && lane == 0) { flags[1] = 1; fail(a.status, 3, t); }
            }
            __syncthreads();  // G1
            if (flags[1]) break;
            // the energy of position rank + 32 wave: v . tanh(q [+ location] + P) + b_v
            // (common_layers.py:166-182), published XCD-locally
            if (rank + 32 * wave < L) {
                float x0 = xq[lane], x1 = xq[lane + 64];
                if (gf & GEN_LOCATION) {
                    x0 += gl0;
                    x1 += gl1;
                }
                const float e = wave_sum_dpp(gv0 * tanh_fast(x0 + gp0) + gv1 * tanh_fast(x1 + gp1));
                if (lane == 0) publish_xcd(a.gran + (t & 1) * GR_TOTAL + s_e + rank + 32 * wave, E + 7, e + vb);
            }
            // every CU gathers the XCD's L energies (waves 0-1: positions 2 pk, 2 pk + 1)
            if (wave < 2) {
                for (int i = 0; i < a.sleep_e; ++i) __builtin_amdgcn_s_sleep(1);
                const int p0 = 2 * pk;
                float e0 = 0.f, e1 = 0.f;
                const bool ok =
                    sweep_pair(rg, p0 < L ? s_e + (t & 1) * GR_TOTAL + p0 : -1, p0 + 1 < L, E + 7, e0, e1, tmo);
                geg[p0] = e0;
                geg[p0 + 1] = e1;
                if (!ok && lane == 0) { flags[1] = 1; fail(a.status, 8, t); }
            }
            __syncthreads();  // G2
            if (flags[1]) break;
            RES_MARK(6);
            // the weights over all L positions, identically in every wave of every CU: lane holds
            // positions ps[i] = (i >> 1) 128 + 2 lane + (i & 1), reductions are DPP wave reductions
            const float* wold = gw + (t & 1) * GW_PAD + 16;  // previous step's weights (position j at j)
            float* wnew = gw + ((t & 1) ^ 1) * GW_PAD + 16;
            int ps[4];
            bool in[4];
            float e[4];
            {
                const float2 g0 = *reinterpret_cast<const float2*>(geg + 2 * lane);
                const float2 g1 = *reinterpret_cast<const float2*>(geg + 128 + 2 * lane);
                e[0] = g0.x; e[1] = g0.y; e[2] = g1.x; e[3] = g1.y;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                ps[i] = (i >> 1) * 128 + 2 * lane + (i & 1);
                in[i] = ps[i] < L;
                if (!in[i]) e[i] = -INFINITY;
            }
            if (gf & GEN_WINDOW) {
                // eval windowing (common_layers.py:184-197)
                const int back = gwin - 2, front = gwin + 6;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (in[i] && ((back > 0 && ps[i] < back) || (front < L && ps[i] >= front))) e[i] = -INFINITY;
                if (gwin == -1) {
                    const float m = wave_max_dpp(fmaxf(fmaxf(e[0], e[1]), fmaxf(e[2], e[3])));
                    if (lane == 0) e[0] = m;
                }
                float bv = e[0];
                int bi = ps[0];
#pragma unroll
                for (int i = 1; i < 4; ++i)
                    if (e[i] > bv) { bv = e[i]; bi = ps[i]; }
                wave_argmax(bv, bi);
                gwin = __builtin_amdgcn_readfirstlane(bi);
            }
            // normalisation (common_layers.py:239-245)
            float al[4];
            if (gf & GEN_SOFTMAX) {
                const float m = wave_max_dpp(fmaxf(fmaxf(e[0], e[1]), fmaxf(e[2], e[3])));
#pragma unroll
                for (int i = 0; i < 4; ++i) al[i] = in[i] ? expf(e[i] - m) : 0.f;
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) al[i] = in[i] ? sigmoidf_(e[i]) : 0.f;
            }
            {
                const float S = wave_sum_dpp((al[0] + al[1]) + (al[2] + al[3]));
#pragma unroll
                for (int i = 0; i < 4; ++i) al[i] = al[i] / S;
            }
            if ((gf & GEN_LOCATION) && wave == 0) {  // update_location_attention (:163-164), own lanes' positions
                float2* c01 = reinterpret_cast<float2*>(gcum + 16 + 2 * lane);
                float2* c23 = reinterpret_cast<float2*>(gcum + 16 + 128 + 2 * lane);
                const float2 o01 = *c01, o23 = *c23;
                *c01 = float2{o01.x + al[0], o01.y + al[1]};
                *c23 = float2{o23.x + al[2], o23.y + al[3]};
            }
            float w[4];
            if (gf & GEN_FORWARD) {
                // apply_forward_attention (:199-223); wold[-1] is the zero pad
                float an[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float ao = wold[ps[i]], pv = wold[ps[i] - 1];
                    const float mix = __fadd_rn(__fadd_rn(__fmul_rn(1.f - gu, ao), __fmul_rn(gu, pv)), 1e-8f);
                    an[i] = in[i] ? __fmul_rn(mix, al[i]) : 0.f;
                }
                if (gf & GEN_MASK) {
                    // eval mask (:207-213), Python slicing incl. the negative-index wrap for n < 2
                    const float rmax = wave_max_dpp(fmaxf(fmaxf(in[0] ? an[0] : -INFINITY, in[1] ? an[1] : -INFINITY),
                                                          fmaxf(in[2] ? an[2] : -INFINITY, in[3] ? an[3] : -INFINITY)));
                    const int cx = gn >= 2 ? gn - 2 : gn - 2 + L, lo = gn >= 1 ? gn - 1 : L - 1;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const bool keep = in[i] && ps[i] < gn + 3 && ps[i] >= lo;
                        an[i] = ps[i] == cx ? 0.01f * rmax : (keep ? an[i] : 0.f);
                    }
                }
                const float denom = wave_sum_dpp((an[0] + an[1]) + (an[2] + an[3]));
#pragma unroll
                for (int i = 0; i < 4; ++i) w[i] = in[i] ? an[i] / denom : 0.f;
                if (gf & GEN_MASK) {
                    // next n = argmax(prev_alpha) = 1 + first argmax of alpha[0..L-2] (0 when all zero)
                    float bv = -1.f;
                    int bi = 0x7fffffff;
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (ps[i] <= L - 2 && w[i] > bv) { bv = w[i]; bi = ps[i]; }
                    wave_argmax(bv, bi);
                    gn = __builtin_amdgcn_readfirstlane(bv > 0.f ? bi + 1 : 0);
                }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) w[i] = al[i];
            }
            RES_MARK(7);
            const float tail = wave_sum_dpp(((ps[0] >= L - 2 && in[0] ? w[0] : 0.f) + (ps[1] >= L - 2 && in[1] ? w[1] : 0.f)) +
                                            ((ps[2] >= L - 2 && in[2] ? w[2] : 0.f) + (ps[3] >= L - 2 && in[3] ? w[3] : 0.f)));
            // context of this CU's channels (bmm, :217 / :253), published XCD-locally with the tail
            float c0 = 0.f, c1 = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                c0 = fmaf(w[i], gen_e[i].x, c0);
                c1 = fmaf(w[i], gen_e[i].y, c1);
            }
            c0 = wave_sum_dpp(c0);
            c1 = wave_sum_dpp(c1);
            {
                u64* gcx = Gc + (t & 1) * GR_TOTAL;
                if (lane < 2) publish_xcd(gcx + 16 * rank + 2 * wave + lane, E + 4, lane ? c1 : c0);
                if (rank == 0 && wave == 0 && lane == 2) publish_xcd(gcx + ENC, E + 4, tail);
            }
            if (tid == 0) { RES_EV(t, 11) }
            RES_MARK(8);
            // this step's weights (next step's previous alpha / location input), cumulative weights,
            // alignment row (tacotron2.py:262-266)
            if (wave == 0) {
                *reinterpret_cast<float2*>(wnew + 2 * lane) = float2{w[0], w[1]};
                *reinterpret_cast<float2*>(wnew + 128 + 2 * lane) = float2{w[2], w[3]};
                if (xlog && rank == 0 && t < a.hist_cap) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (ps[i] < a.Lalign) a.align_hist[(int64_t)t * a.Lalign + ps[i]] = w[i];
                }
            }
        }
        if (att_cu) {
            const float* aold = abuf + (t & 1) * RES_LMAX;
            float* anew = abuf + ((t & 1) ^ 1) * RES_LMAX;
            float* candv = scr + 2 * RES_WAVES;
            const int cx = n >= 2 ? n - 2 : n - 2 + L, clo = n >= 1 ? n - 1 : L - 1, chi = min(n + 2, L - 1);
            // candidate slot s = tid / 32 (32 lanes x 4 dims): its operands that do not depend on
            // the query are read before the query arrives
            const int sl = tid >> 5, sub = tid & 31;
            const int pos = t > 0 ? res_candidate(sl, n, n_prev, L) : -1;
            float xvd[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) xvd[m] = xv[sub + 32 * m];
            const float a_pos = pos >= 0 ? aold[pos] : 0.f, a_prev = pos > 0 ? aold[pos - 1] : 0.f;
            if (wave < 2) {  // query row pk = its two half-rows
                for (int i = 0; i < a.sleep_q; ++i) __builtin_amdgcn_s_sleep(1);
                float q0, q1;
                const bool ok = sweep_pair(rg, s_q + (t & 1) * GR_TOTAL + 2 * pk, true, E + 3, q0, q1, tmo);
                xq[pk] = q0 + q1;
                if (!ok && lane == 0) { flags[1] = 1; fail(a.status, 3, t); }
            }
            __syncthreads();  // A1
            if (tid == 0) { RES_EV(t, 9) }
            if (flags[1]) break;
            RES_MARK(6);
            bool full = t == 0;
            float rm = -INFINITY, cand = -INFINITY;
            if (!full) {
                float part = 0.f;
#pragma unroll
                for (int m = 0; m < 4; ++m) part += xvd[m] * tanh_fast(xq[sub + 32 * m] + ptc[m]);
                const float e = sum32_dpp(part);
                if (sub == 31) {
                    float v = -INFINITY;
                    if (pos >= 0) {
                        const float sg = sigmoid_fast(e + vb);
                        const float mix = __fadd_rn(__fadd_rn(__fmul_rn(1.f - ufa, a_pos), __fmul_rn(ufa, a_prev)), 1e-8f);
                        v = __fmul_rn(mix, sg);
                        an[pos] = v;
                    }
                    candv[sl] = v;
                }
                __syncthreads();  // A2
                if (tid == 0) { RES_EV(t, 10) }
                RES_MARK(14);
                // one LDS read per lane (slot lane % 16), the max by DPP, the window slots 1-4 by
                // readlane below: no chain of dependent LDS reads
                cand = candv[lane & 15];
                rm = wave_max_dpp(cand);
                full = !(rm >= 1e-8f);  // uniform
            }
            if (full) {
                // every position: wave w owns dims [16w, 16w + 16), lanes own positions
                float xqd[16];
#pragma unroll
                for (int dd = 0; dd < 16; ++dd) xqd[dd] = xq[16 * wave + dd];
#pragma unroll 1
                for (int jj = lane; jj < L; jj += 64) {
                    float s = 0.f;
#pragma unroll
                    for (int dd = 0; dd < 16; ++dd) {
                        const int d = 16 * wave + dd;
                        s += xv[d] * tanh_fast(xqd[dd] + a.Pt[(int64_t)d * a.Lcap + jj]);
                    }
                    red[wave * RES_LMAX + jj] = s;
                }
                __syncthreads();
                const int j = tid;
                float anj = -INFINITY;
                if (j < L) {
                    float e = 0.f;
#pragma unroll
                    for (int w = 0; w < RES_WAVES; ++w) e += red[w * RES_LMAX + j];
                    const float sg = sigmoid_fast(e + vb);
                    const float prev = j > 0 ? aold[j - 1] : 0.f;
                    const float mix = __fadd_rn(__fadd_rn(__fmul_rn(1.f - ufa, aold[j]), __fmul_rn(ufa, prev)), 1e-8f);
                    anj = __fmul_rn(mix, sg);
                    an[j] = anj;
                }
                const float wmax = wave_max_dpp(anj);
                if (lane == 0) scr[2 * wave + 1] = wmax;
                __syncthreads();
                rm = -INFINITY;
#pragma unroll
                for (int k = 0; k < RES_WAVES; ++k) rm = fmaxf(rm, scr[2 * k + 1]);
            }
            RES_MARK(7);
            // the surviving window [n-1, n+2] without (n-2) mod L: its unnormalised weights once
            // the surviving window's unnormalised weights: candidate slots 1-4 hold exactly an[clo + k]
            // (the same lane wrote both); the full-L path reads them from an[]
            float aw[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float c = full ? an[clo + k] : __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cand), 1 + k));
                aw[k] = (clo + k <= chi && clo + k != cx) ? c : 0.f;
            }
            const float rs = ((aw[0] + aw[1]) + aw[2]) + aw[3];  // index order
            const float vx = 0.01f * rm;  // alpha[n-2] = 0.01 * val
            const float denom = rs + vx;
            const float inv = 1.f / denom;
            const float wcx = vx * inv;
            float ww[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) ww[k] = aw[k] * inv;
            auto weight = [&](int p) -> float {
                if (p == cx) return wcx;
                return (p >= clo && p <= chi) ? ww[p - clo] : 0.f;
            };
            const float tail = weight(L - 2) + weight(L - 1);  // tacotron2.py:268
            float bv = 0.f;
            int bi = -1;
            auto consider = [&](int p) {
                const float wp = weight(p);
                if (p <= L - 2 && wp > bv) { bv = wp; bi = p; }
            };
            if (cx < clo) consider(cx);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (clo + k <= chi) consider(clo + k);
            if (cx > chi) consider(cx);
            float ctx = 0.f;
            if (cx < clo) ctx += wcx * ex;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (clo + k <= chi) ctx += (clo + k == cx ? wcx * ex : ww[k] * erow[k]);
            if (cx > chi) ctx += wcx * ex;
            RES_MARK(15);
            publish_xcd(Gc + (t & 1) * GR_TOTAL + tid, E + 4, ctx);
            if (tid == 0) publish_xcd(Gc + (t & 1) * GR_TOTAL + ENC, E + 4, tail);
            xctx[tid] = ctx;  // this CU skips the gather
            if (tid == 0) xctx[ENC] = tail;
            if (tid == 0) { RES_EV(t, 11) }
            RES_MARK(8);
            // off the critical path: this step's alpha (next step's prev_alpha) and alignment row
            wdef = tid < L ? weight(tid) : 0.f;
            n_prev = n;
            n = bi >= 0 ? bi + 1 : 0;  // argmax(prev_alpha) of the next step (its loads: h_att wait)
            // the deferred decoder-LSTM h_att half is on this CU's h_dec path: four chunks' LDS
            // operands in flight at a time (the two-chunk loop waited out eight LDS round trips)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float4 wv[4], xv4[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    wv[j] = wdl[((4 * h + j) * 16 + r) * 32 + ks];
                    xv4[j] = ld4(xh_att + (4 * h + j) * 128 + ks * 4);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) acc_d = dot4(wv[j], xv4[j], acc_d);
                asm volatile("" ::: "memory");
            }
            RES_MARK(9);
        }
        // this wave's prenet-1 row weights (step 11) from the XCD's L2, in flight while the context
        // (and then h_dec) is awaited
        float4 w1[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) w1[i] = ld4(w1p + i * 256);
        // 8) gather ctx_t and the tail
        if (wave < 5 && !att_cu) {  // waves 0-3: the 512 context values as pairs; wave 4, lane 0: the tail
            const int gc = s_c + (t & 1) * GR_TOTAL;
            for (int i = 0; i < a.sleep_ctx; ++i) __builtin_amdgcn_s_sleep(4);
            float c0 = 0.f, c1 = 0.f;
            const bool ok = wave < 4 ? sweep_pair(rg, gc + 2 * pk, true, E + 4, c0, c1, tmo)
                                     : sweep_pair(rg, lane == 0 ? gc + ENC : -1, false, E + 4, c0, c1, tmo);
            if (wave < 4) {
                xctx[2 * pk] = c0;
                xctx[2 * pk + 1] = c1;
            } else if (lane == 0) {
                xctx[ENC] = c0;
            }
            if (!ok && lane == 0) { flags[1] = 1; fail(a.status, 4, t); }
        }
        __syncthreads();  // B4
        if (tid == 0) { RES_EV(t, 4) }
        if (flags[1]) break;
        RES_MARK(10);
        // 9) context part, cell
#pragma unroll
        for (int i = 0; i < 4; ++i) acc_d = dot4(wdc[i], ld4(xctx + i * 128 + ks * 4), acc_d);
        acc_d = sum32_dpp(acc_d);
        if (ks == 31) gates[r] = acc_d;
        __syncthreads();  // B5
        RES_MARK(11);
        if (tid < 16) {
            float cs = st[36 + (tid & 3)];
            const float h = lstm_cell16(gates[tid] + st[16 + tid], cs);
            if (tid < 4) {
                st[36 + tid] = cs;
                st[44 + tid] = h;
                publish(G + GR_HDEC + 4 * c + tid, E + 5, h);
                if (tid == 0) { RES_EV(t, 5) }
            }
        }
        if constexpr (GEN) {
            // off the critical path (the h_dec edge is in flight): the transition agent's wave
            // partials of u = sigmoid(ta([ctx_t, h_att_t])) for the next step (common_layers.py:220-222)
            // and the next step's location features (its input is this step's weights)
            if (gf & GEN_TA) {
                float pta = 0.f;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const int idx = 3 * tid + k;
                    pta = fmaf(gtw[k], idx < ENC ? xctx[idx] : xh_att[idx - ENC], pta);
                }
                pta = wave_sum_dpp(pta);
                if (lane == 0) gts[wave] = pta;
            }
            if (gf & GEN_LOCATION) gen_location(gw + ((t & 1) ^ 1) * GW_PAD);
        }
        // the attention CU's alpha (next step's prev_alpha) and alignment row, after its h_dec
        // publish: the eight attention CUs are the h_dec edge's last publishers
        if (att_cu) {
            float* anew = abuf + ((t & 1) ^ 1) * RES_LMAX;
            if (tid < L) anew[tid] = wdef;
            if (att_log && t < a.hist_cap && tid < a.Lalign) a.align_hist[(int64_t)t * a.Lalign + tid] = wdef;
        }
        // 10) gather h_dec_t
        {
            for (int i = 0; i < a.sleep_hdec; ++i) __builtin_amdgcn_s_sleep(4);
            float h0, h1;
            const bool ok = sweep_pair(rg, (t & 1) * GR_TOTAL + GR_HDEC + 2 * pk, true, E + 5, h0, h1, tmo);
            xh_dec[2 * pk] = h0;
            xh_dec[2 * pk + 1] = h1;
            if (!ok && lane == 0) { flags[1] = 1; fail(a.status, 5, t); }
        }
        __syncthreads();  // B6
        if (tid == 0) { RES_EV(t, 6) }
        if (flags[1]) break;
        if constexpr (GEN) {
            if (gf & GEN_TA) {
                float sta = gts[0];
#pragma unroll
                for (int k = 1; k < RES_WAVES; ++k) sta += gts[k];
                gu = sigmoidf_(sta + gtb);
            }
        }
        RES_MARK(12);
        long long m0 = 0;  // prenet-1 / mel / stop row phase timing (wave 2, lane 0)
        if (prof && tid == 128) m0 = (long long)wall_clock64();
        // 11) this wave's folded prenet-1 row of step t+1 (XCD copy) and, on the stop CU's wave 3,
        //     the stop row in the same pass
        {
            const bool stw = stop_cu && wave == 3;
            const float4* wsr = reinterpret_cast<const float4*>(rm) + 6 * 64 + lane;
            float s = 0.f, ss = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float4 x = ld4(xh_dec + i * 256 + lane * 4);
                s = dot4(w1[i], x, s);
                if (stw) ss = dot4(wsr[i * 64], x, ss);
            }
#pragma unroll
            for (int i = 4; i < 6; ++i) {
                const float4 x = ld4(xctx + (i - 4) * 256 + lane * 4);
                s = dot4(w1[i], x, s);
                if (stw) ss = dot4(wsr[i * 64], x, ss);
            }
            s = wave_sum_dpp(s);
            u64* g1 = G1 + (t & 1) * GR_TOTAL;
            if (has_row && lane == 0) {
                const float p = fmaxf(s + bp1, 0.f);
                publish_xcd(g1 + r0, E + 6, p);
                if (wave == 0) { RES_EV(t, 7) }
                if (xlog) a.pre1[r0] = p;  // the next step's layer 1 (continuous mode reads it)
            }
            if (stw) {
                ss = wave_sum_dpp(ss);
                if (lane == 0) {
                    // stopnet + stop rule (tacotron2.py:219-224, 257-277), as EPI_MEL_FUSED rule 0;
                    // every XCD's stop CU decides identically, the logging XCD writes the outputs
                    const float stv = sigmoidf_(ss + st[49]);
                    if (xlog && t < a.hist_cap) a.stop_hist[t] = stv;
                    const float tail = xctx[ENC];
                    int* sst = reinterpret_cast<int*>(st);
                    const int f1 = sst[50] | ((tail > 0.8f && t > L) ? 1 : 0);
                    sst[50] = f1;
                    int nd = 0;
                    if (f1 && t > 2 * L) {
                        sst[51] += 1;
                        if (sst[51] > 20) nd = 1;
                    } else if (t + 1 == a.max_steps) {
                        nd = 1;
                    }
                    if (!nd && t + 1 >= a.hist_cap) {  // cannot happen: the rule stops by max_steps + 20
                        nd = 1;
                        fail(a.status, 100);
                    }
                    if (nd && xlog) {
                        a.done[0] = 1;
                        a.n_steps[0] = t + 1;
                    }
                    publish_xcd(g1 + PRE, E + 6, nd ? 0.f : 1.f);
                }
            }
        }
        if (prof && tid == 128) pacc[13] += (long long)wall_clock64() - m0;
    }
    if (flags[1]) return;
    if (wave == 4 && t > 0) mel_row(t - 1);  // the last step's mel row (its h_att gather never came)
    if (prof && tid == 0)
        for (int k = 0; k < RES_PHASES; ++k) a.prof[(c == 0 ? 0 : 1) * RES_PHASES + k] = pacc[k];
    // the last step t-1 leaves its state where the multi-launch path's would be
    const int pl = (t - 1) & 1;
    if (tid < 4) {
        a.h_att[pl * a.hps + 4 * c + tid] = st[40 + tid];
        a.c_att[4 * c + tid] = st[32 + tid];
        a.h_dec[pl * a.hps + 4 * c + tid] = st[44 + tid];
        a.c_dec[4 * c + tid] = st[36 + tid];
    }
    if (c == 0)
        for (int k = tid; k < ENC; k += RES_THREADS) a.xa[(1 - pl) * a.xps + PRE + k] = xctx[k];
}

// ---- weight packing (once, at tts_decoder_create)
__global__ void res_pack_wa(const float* wih, const float* whh, float4* out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)RES_CUS * 14 * RES_THREADS) return;
    const int tid = idx % RES_THREADS, i4 = (idx / RES_THREADS) % 14, c = idx / (14 * RES_THREADS);
    const int r = tid >> 5, ks = tid & 31, row = (r >> 2) * HATT + 4 * c + (r & 3);
    float v[4];
    for (int j = 0; j < 4; ++j) {
        const int k = i4 * 128 + ks * 4 + j;  // over [prenet 256 | ctx 512 | h_att 1024]
        v[j] = k < XA ? wih[(int64_t)row * XA + k] : whh[(int64_t)row * HATT + (k - XA)];
    }
    out[idx] = float4{v[0], v[1], v[2], v[3]};
}
__global__ void res_pack_wd(const float* wih, const float* whh, float4* wdl, float4* wdc) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    constexpr int PER = 16 * 16 * 32 + 4 * RES_THREADS;  // float4 per CU: LDS image + ctx part
    if (idx >= (int64_t)RES_CUS * PER) return;
    const int c = idx / PER, e = idx % PER;
    float v[4];
    if (e < 16 * 16 * 32) {
        const int i4 = e / 512, r = (e / 32) % 16, ks = e % 32;
        const int row = (r >> 2) * HDEC + 4 * c + (r & 3);
        for (int j = 0; j < 4; ++j) {
            const int k = i4 * 128 + ks * 4 + j;  // over [h_att 1024 | h_dec 1024]
            v[j] = k < HATT ? wih[(int64_t)row * (HATT + ENC) + k] : whh[(int64_t)row * HDEC + (k - HATT)];
        }
        wdl[(int64_t)c * 8192 + e] = float4{v[0], v[1], v[2], v[3]};
    } else {
        const int f = e - 16 * 16 * 32, i4 = f / RES_THREADS, tid = f % RES_THREADS;
        const int r = tid >> 5, ks = tid & 31, row = (r >> 2) * HDEC + 4 * c + (r & 3);
        for (int j = 0; j < 4; ++j) v[j] = wih[(int64_t)row * (HATT + ENC) + HATT + i4 * 128 + ks * 4 + j];
        wdc[((int64_t)c * 4 + i4) * RES_THREADS + tid] = float4{v[0], v[1], v[2], v[3]};
    }
}
__global__ void res_pack_bias(const float* abih, const float* abhh, const float* dbih, const float* dbhh, float* ba,
                              float* bd) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx < RES_CUS * 16) {
        const int c = idx / 16, r = idx % 16, row = (r >> 2) * HATT + 4 * c + (r & 3);
        ba[idx] = abih[row] + abhh[row];
        bd[idx] = dbih[row] + dbhh[row];
    }
}

__global__ void res_pack_loc(const float* w, float* out) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // out [2 c][NLOC f][32 k], k = 31 zero
    if (idx >= 2 * NLOC * 32) return;
    const int k = idx & 31, f = (idx >> 5) % NLOC, c = idx / (32 * NLOC);
    out[idx] = k < KLOC ? w[(f * 2 + c) * KLOC + k] : 0.f;
}

}  // namespace

hipError_t resident_pack_location(const float* w, float* out, hipStream_t s) {
    hipLaunchKernelGGL(res_pack_loc, dim3((2 * NLOC * 32 + 255) / 256), dim3(256), 0, s, w, out);
    return hipGetLastError();
}

void resident_weight_floats(size_t* wa, size_t* wdl, size_t* wdc) {
    *wa = (size_t)RES_CUS * 14 * RES_THREADS * 4;
    *wdl = (size_t)RES_CUS * 16 * 16 * 32 * 4;
    *wdc = (size_t)RES_CUS * 4 * RES_THREADS * 4;
}

hipError_t resident_pack(const ResSrc& s, const ResWeights& w, hipStream_t st) {
    auto blocks = [](int64_t n) { return dim3((unsigned)((n + 255) / 256)); };
    hipLaunchKernelGGL(res_pack_wa, blocks((int64_t)RES_CUS * 14 * RES_THREADS), dim3(256), 0, st, s.a_wih, s.a_whh,
                       w.wa);
    hipLaunchKernelGGL(res_pack_wd, blocks((int64_t)RES_CUS * (8192 + 4 * RES_THREADS)), dim3(256), 0, st, s.d_wih,
                       s.d_whh, w.wdl, w.wdc);
    (void)hipMemcpyAsync(w.w2, s.w_pre2, sizeof(float) * PRE * PRE, hipMemcpyDeviceToDevice, st);
    if (s.b_pre2)
        (void)hipMemcpyAsync(w.b2, s.b_pre2, sizeof(float) * PRE, hipMemcpyDeviceToDevice, st);
    else
        (void)hipMemsetAsync(w.b2, 0, sizeof(float) * PRE, st);
    (void)hipMemcpyAsync(w.wq, s.w_q, sizeof(float) * ADIM * HATT, hipMemcpyDeviceToDevice, st);
    (void)hipMemcpyAsync(w.wf, s.wf, sizeof(float) * s.nrows * (HDEC + ENC), hipMemcpyDeviceToDevice, st);
    (void)hipMemcpyAsync(w.bf, s.bf, sizeof(float) * s.nrows, hipMemcpyDeviceToDevice, st);
    hipLaunchKernelGGL(res_pack_bias, blocks(RES_CUS * 16), dim3(256), 0, st, s.a_bih, s.a_bhh, s.d_bih, s.d_bhh, w.ba,
                       w.bd);
    return hipGetLastError();
}

size_t resident_smem_bytes() { return (size_t)SM_FLOATS * sizeof(float); }

hipError_t resident_prepare() {
    const void* fns[] = {reinterpret_cast<const void*>(&resident_decoder_kernel<false, false>),
                         reinterpret_cast<const void*>(&resident_decoder_kernel<true, false>),
                         reinterpret_cast<const void*>(&resident_decoder_kernel<false, true>),
                         reinterpret_cast<const void*>(&resident_decoder_kernel<true, true>)};
    for (const void* fn : fns) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)resident_smem_bytes());
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_resident(const ResArgs& a, hipStream_t s, bool* launched) {
    *launched = false;
    if (a.L < 2 || a.L > RES_LMAX || a.nmel > RES_CUS || a.nmel + PRE + 1 != a.nrows) return hipErrorInvalidValue;
    ResArgs arg = a;
    void* args[] = {&arg};
    if (a.gen && ((a.gen & GEN_TA) && !(a.ta_w && a.ta_b))) return hipErrorInvalidValue;
    if (a.gen && ((a.gen & GEN_LOCATION) && !(a.att_w0 && a.att_cum0 && a.loc_conv && a.loc_dense)))
        return hipErrorInvalidValue;
    if (a.gen && (a.gen & GEN_WINDOW) && !a.win0) return hipErrorInvalidValue;
    const void* fn = a.gen ? (a.prof ? reinterpret_cast<const void*>(&resident_decoder_kernel<true, true>)
                                     : reinterpret_cast<const void*>(&resident_decoder_kernel<false, true>))
                           : (a.prof ? reinterpret_cast<const void*>(&resident_decoder_kernel<true, false>)
                                     : reinterpret_cast<const void*>(&resident_decoder_kernel<false, false>));
    return launch_persistent(fn, dim3(RES_CUS), dim3(RES_THREADS), args, resident_smem_bytes(), s, launched);
}

}  // namespace tts

// Resident decoder for small batches: the whole decoder loop of Decoder.inference
// (layers/tacotron2.py:249-285) for up to RB_MAXB sentences as ONE persistent launch, each sentence
// with the per-sentence semantics of a batch-1 run (the reference's stop rule is batch-1).
//
// Weight-stationary like the batch-1 kernel (resident.h): 256 workgroups, one per compute unit,
// each holding its 16 gate rows of both LSTMs (units 4c..4c+3) for the whole launch, so a step
// streams no weights; the step's cost is its hand-offs, which now carry every sentence's values.
// Where the weights live differs: the batch-1 kernel keeps the decoder LSTM's recurrent half in
// LDS (128 KiB), which here holds the batch's activations (h_att, h_dec, context, prenet rows), so
// BOTH LSTMs' rows sit in the register file.  That is 272 KiB per CU, more than half of it, so a
// workgroup is 4 waves (one per SIMD): a wave then owns 512 registers (VGPRs + AGPRs, the compiler
// keeping what the VALU does not need at the moment in AGPRs); at 2 waves per SIMD (the batch-1
// layout) a wave owns 256 and the weights left no room for the rest of the step.
//
// LSTM layout: wave w owns unit u = w (4 units per CU) and lane l the k-slice l of 64, holding the
// 4 gates over its slice (attention LSTM: prenet 4 + ctx 8 + h_att 16 k; decoder LSTM: h_att 16 +
// ctx 8 + h_dec 16 k; 272 weight registers): one LDS read of an activation feeds 4 FMAs, and the
// NB sentences reuse every weight.  The 4 NB partial sums per lane are reduced over the wave by a
// transpose reduction (value count halving per xor level), fixed orders throughout (bitwise
// run-to-run deterministic); the unit's cell then runs in the same wave, no workgroup barrier.
//
// Per-sentence work stays XCD-local as in the batch-1 kernel: every XCD computes its own copy of
// prenet-2, the query, the attention and the prenet-1 / stop rows for all sentences.  The attention
// of sentence b runs in wave b of every CU of the XCD: energies of positions rank + 32 i, exchanged
// XCD-locally, the normalisation / forward attention / mask over all positions inside that one wave,
// then the context of the CU's 16 channels.  Two device-wide edges per step (h_att, h_dec).
//
// Scope: 2 <= B <= RB_MAXB per launch (a larger request runs consecutive launches), every
// L_b <= 256, nmel <= 256, the attention configurations without location features, windowing or
// transition agent (forward attention with or without the eval mask, sigmoid or softmax:
// synthesize.py's and Synthesizer.tts()'s); the others run multi-launch.
#include "handoff.h"
#include "resident.h"

namespace tts {
namespace {
using namespace handoff;

constexpr int RB_THREADS = 256;
constexpr int GW_PAD = RES_LMAX + 32;  // previous weights, zero-padded by 16 on both sides
constexpr int KA = 28, KD = 40;        // k per lane: attention LSTM, decoder LSTM

// granule slots (u64) of one step parity
constexpr int RBG_HATT = 0;                           // [RB_MAXB][1024] device-wide
constexpr int RBG_HDEC = RBG_HATT + RB_MAXB * HATT;   // [RB_MAXB][1024] device-wide
constexpr int RBG_SETUP = RBG_HDEC + RB_MAXB * HDEC;  // [256] XCD ids (parity 0)
constexpr int RBG_X = RBG_SETUP + 256;                // per-XCD blocks of RBX_SIZE:
constexpr int RBX_PRE2 = 0;                           //   prenet-2 [RB_MAXB][256]
constexpr int RBX_Q = RBX_PRE2 + RB_MAXB * PRE;       //   query [RB_MAXB][128]
constexpr int RBX_E = RBX_Q + RB_MAXB * ADIM;         //   energies [RB_MAXB][256]
constexpr int RBX_CTX = RBX_E + RB_MAXB * RES_LMAX;   //   context [RB_MAXB][512]
constexpr int RBX_TAIL = RBX_CTX + RB_MAXB * ENC;     //   stop-rule tails [RB_MAXB] (16 slots)
constexpr int RBX_P1 = RBX_TAIL + 16;                 //   prenet-1 rows [RB_MAXB][256]
constexpr int RBX_FLAG = RBX_P1 + RB_MAXB * PRE;      //   continue flags [RB_MAXB] (16 slots)
constexpr int RBX_SIZE = RBX_FLAG + 16;
constexpr int RBG_TOTAL = RBG_X + 8 * RBX_SIZE;
static_assert(RBX_SIZE % 16 == 0 && RBG_X % 16 == 0, "pair loads need 16-byte aligned blocks");
static_assert(RB_MAXB <= 4 && RB_MAXB % 2 == 0, "one attention wave per sentence; flags read in pairs");

template <int NB>
struct Lds {
    static constexpr int XHATT = 0;
    static constexpr int XHDEC = XHATT + NB * HATT;
    static constexpr int XCTX = XHDEC + NB * HDEC;
    static constexpr int XTAIL = XCTX + NB * ENC;
    static constexpr int XPRE = XTAIL + 16;
    static constexpr int XP1 = XPRE + NB * PRE;
    static constexpr int GW = XP1 + NB * PRE;              // [NB][2][GW_PAD]
    static constexpr int GSUM = GW + NB * 2 * GW_PAD;      // [4 units][4 NB]
    static constexpr int RM = GSUM + 4 * 4 * NB;           // mel row c [6][64] float4 + stop row [6][64] float4
    static constexpr int INTS = RM + 2 * 6 * 64 * 4;       // [0, 8) flags, [8, 16) active, [16, 24) flag1, [24, 32) count
    static constexpr int ENC_L = NB == 2 ? RES_LMAX : 128;  // positions of the context channels held in LDS
    static constexpr int ENCS = INTS + 32;                 // [NB][ENC_L][16] the CU's context channels
    static constexpr int WDC = ENCS + NB * ENC_L * 16;     // [8][256 threads] float4: decoder LSTM ctx part
    static constexpr int WQ = WDC + 8 * RB_THREADS * 4;    // [4 waves][1024] the waves' query rows
    static constexpr int TOTAL = WQ + 4 * HATT;
};

// The transpose reduction: V values per lane summed over the 64 lanes of the wave; lane l ends with
// the total of value index l >> (6 - log2 V).  Each level halves the values a lane keeps: it keeps
// one half and adds its partner's copy of the same half.  No LDS crossbar: the 32- and 16-lane
// levels are gfx950's v_permlane32_swap / v_permlane16_swap (one instruction exchanges a value pair
// between the two halves), the lower ones DPP (row_ror:8, row_half_mirror, quad_perm xor 2 / xor 1;
// the half mirror pairs lane i with 7 - i, opposite in bit 2 and equal above it, which is all the
// reduction needs).  (Lane selects by bit masks, not `up ? v[i] : v[h + i]`: the compiler turns a
// select of two array elements into a select of their addresses, which sends the array to scratch.)
template <int M>
__device__ __forceinline__ float xpartner(float x) {
    static_assert(M == 8 || M == 4 || M == 2 || M == 1, "DPP levels");
    return M == 8 ? dpp_move<0x128, 0xf>(x, 0.f)    // row_ror:8
         : M == 4 ? dpp_move<0x141, 0xf>(x, 0.f)    // row_half_mirror
         : M == 2 ? dpp_move<0x4E, 0xf>(x, 0.f)     // quad_perm [2,3,0,1]
                  : dpp_move<0xB1, 0xf>(x, 0.f);    // quad_perm [1,0,3,2]
}
// lanes with bit M clear keep lo, the others hi; returns keep + the partner's copy of it
template <int M>
__device__ __forceinline__ float xlevel(float lo, float hi) {
    if constexpr (M == 32 || M == 16) {
        const auto r = M == 32 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(lo), __float_as_uint(hi), false, false)
                               : __builtin_amdgcn_permlane16_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
        return __uint_as_float(r[0]) + __uint_as_float(r[1]);
    } else {
        const unsigned msk = (threadIdx.x & M) ? 0xffffffffu : 0u;
        const unsigned l = __float_as_uint(lo), h = __float_as_uint(hi);
        const float send = __uint_as_float((l & msk) | (h & ~msk));
        const float keep = __uint_as_float((h & msk) | (l & ~msk));
        return keep + xpartner<M>(send);
    }
}
template <int LEV, int V>
__device__ __forceinline__ void xstep(float (&v)[V]) {
    constexpr int M = 32 >> LEV;
    constexpr int H = (V >> LEV) >> 1;
    if constexpr (H >= 1) {
#pragma unroll
        for (int i = 0; i < H; ++i) v[i] = xlevel<M>(v[i], v[H + i]);
    } else {
        v[0] = xlevel<M>(v[0], v[0]);  // one value left: a plain butterfly sum
    }
}
template <int V>
__device__ __forceinline__ float xreduce(float (&v)[V]) {
    static_assert(V == 1 || V == 2 || V == 4 || V == 8 || V == 16 || V == 32, "power of two");
    xstep<0>(v);
    xstep<1>(v);
    xstep<2>(v);
    xstep<3>(v);
    xstep<4>(v);
    xstep<5>(v);
    return v[0];
}

__device__ __forceinline__ void fma4(float4 w, float x, float* acc) {
    acc[0] = fmaf(w.x, x, acc[0]);
    acc[1] = fmaf(w.y, x, acc[1]);
    acc[2] = fmaf(w.z, x, acc[2]);
    acc[3] = fmaf(w.w, x, acc[3]);
}
// 4 gates x 4 consecutive k of one sentence
__device__ __forceinline__ void fma44(const float4* w, float4 x, float* acc) {
    fma4(w[0], x.x, acc);
    fma4(w[1], x.y, acc);
    fma4(w[2], x.z, acc);
    fma4(w[3], x.w, acc);
}
__device__ __forceinline__ float dot4(float4 w, float4 x, float acc) {
    acc = fmaf(w.x, x.x, acc);
    acc = fmaf(w.y, x.y, acc);
    acc = fmaf(w.z, x.z, acc);
    return fmaf(w.w, x.w, acc);
}
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Poll NP consecutive granule pairs from even slot `base` (thread i: pairs i, i + 256, ...): every
// poll issues all of the thread's loads before one wait; the values go to dst[2p], dst[2p + 1]
// once every pair of the wave carries `tag`.  false after the timeout.
template <int NP>
__device__ __forceinline__ bool gather_pairs(__amdgpu_buffer_rsrc_t r, int base, unsigned tag, float* dst, long long tmo,
                                             int first_sleep = 0) {
    static_assert(NP % RB_THREADS == 0, "whole pairs per thread");
    constexpr int MAXP = NP / RB_THREADS;
    const int tid = threadIdx.x;
    long long t_end = 0;
    // (a poll storm from every CU the moment it has published slows the stores it waits for)
    for (int i = 0; i < first_sleep; ++i) __builtin_amdgcn_s_sleep(4);
    for (int spin = 0;; ++spin) {
        u32x4 x[MAXP];
#pragma unroll
        for (int i = 0; i < MAXP; ++i)
            x[i] = __builtin_bit_cast(
                u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (base + 2 * (tid + i * RB_THREADS)) * 8, 0, SC1_VOLATILE));
        bool ok = true;
#pragma unroll
        for (int i = 0; i < MAXP; ++i) ok = ok && x[i].y == tag && x[i].w == tag;
        if (__all(ok)) {
#pragma unroll
            for (int i = 0; i < MAXP; ++i)
                *reinterpret_cast<float2*>(dst + 2 * (tid + i * RB_THREADS)) = float2{__uint_as_float(x[i].x), __uint_as_float(x[i].z)};
            return true;
        }
        if (spin == 0) {
            t_end = (long long)wall_clock64() + tmo;
        } else if ((spin & 31) == 0 && (long long)wall_clock64() > t_end) {
            return false;
        }
    }
}

template <int NB, bool PROF>
__global__ __launch_bounds__(RB_THREADS, 1) void resident_batch_kernel(const ResBatchArgs a) {
    using S = Lds<NB>;
    constexpr int V = 4 * NB;  // partial sums per lane (sentence x gate)
    const int c = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // = the LSTM unit 4c + wave
    extern __shared__ __align__(16) float sm[];
    float* xh_att = sm + S::XHATT;
    float* xh_dec = sm + S::XHDEC;
    float* xctx = sm + S::XCTX;
    float* xtail = sm + S::XTAIL;
    float* xpre = sm + S::XPRE;
    float* xp1 = sm + S::XP1;
    float* gw = sm + S::GW;
    float* gsum = sm + S::GSUM + wave * V;
    float* rm = sm + S::RM;
    int* ints = reinterpret_cast<int*>(sm + S::INTS);
    int* flags = ints;        // [1] abort, [2] rank, [3] nx, [4] logging XCD
    int* act = ints + 8;      // sentence b decodes this step
    int* sflag1 = ints + 16;  // stop rule state (the stop CU)
    int* scount = ints + 24;
    // phase clocks (PROF builds): lane 0 of every wave
    long long ptk[RB_PROF_SLOTS] = {}, tprev = 0;
    int t = 0;
    auto mark = [&](int k) {
        if constexpr (PROF) {
            if (lane == 0) {
                const long long now = (long long)wall_clock64();
                ptk[k] += now - tprev;
                tprev = now;
                // absolute clocks at one step: h_att published / gathered, ctx published, h_dec
                // published / gathered, the step's end
                if (t == RB_PROF_T) {
                    if (k == 4) ptk[13] = now;
                    if (k == 5) ptk[14] = now;
                    if (k == 7) ptk[15] = now;
                    if (k == 10) ptk[16] = now;
                    if (k == 11) ptk[17] = now;
                    if (k == 12) ptk[18] = now;
                }
            }
        }
    };

    // ---- weights (once per launch): the 4 gates at each k of this lane's slice
    float4 wa[KA], wd[KD];
    {
        const float4* p = a.wa + (size_t)c * KA * RB_THREADS + tid;
#pragma unroll
        for (int j = 0; j < KA; ++j) wa[j] = p[(size_t)j * RB_THREADS];
        const float4* q = a.wd + (size_t)c * KD * RB_THREADS + tid;
#pragma unroll
        for (int j = 0; j < KD; ++j)
            if (j < 16 || j >= 24) wd[j] = q[(size_t)j * RB_THREADS];
        // the context part (j = 16..23) lives in LDS: read once per step, in phase 10
        for (int j = 0; j < 8; ++j) reinterpret_cast<float4*>(sm + S::WDC)[j * RB_THREADS + tid] = q[(size_t)(16 + j) * RB_THREADS];
    }
    constexpr int KF = HDEC + ENC;
    if (wave == 1 && c < a.nmel)
        for (int i = 0; i < 6; ++i) reinterpret_cast<float4*>(rm)[i * 64 + lane] = ld4(a.wf + (size_t)c * KF + i * 256 + lane * 4);
    // cell lanes b < NB of wave u: unit 4c + u of sentence b (biases, cell states in registers)
    const bool cell_l = lane < NB;
    float bia[4], bid[4], c_att = 0.f, c_dec = 0.f, h_att_l = 0.f, h_dec_l = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        bia[g] = a.ba[c * 16 + g * 4 + wave];
        bid[g] = a.bd[c * 16 + g * 4 + wave];
    }
    if (cell_l && lane < a.B) {  // (padding sentences b >= B: zero state, no reads past the batch)
        c_att = a.c_att[(size_t)lane * HATT + 4 * c + wave];
        c_dec = a.c_dec[(size_t)lane * HDEC + 4 * c + wave];
    }
    // initial activations (multi-launch layout: step 0 reads slot 1 of h_att / h_dec, xa slot 0)
    for (int k = tid; k < NB * HATT; k += RB_THREADS) {
        const int b = k / HATT, j = k % HATT;
        xh_att[k] = b < a.B ? a.h_att[a.hps + (size_t)b * HATT + j] : 0.f;
        xh_dec[k] = b < a.B ? a.h_dec[a.hps + (size_t)b * HDEC + j] : 0.f;
    }
    for (int k = tid; k < NB * ENC; k += RB_THREADS) {
        const int b = k / ENC, j = k % ENC;
        xctx[k] = b < a.B ? a.xa[(size_t)b * XA + PRE + j] : 0.f;
    }
    if (tid < NB) {
        act[tid] = tid < a.B ? 1 : 0;
        sflag1[tid] = tid < a.B ? a.flag1[tid] : 0;
        scount[tid] = tid < a.B ? a.count[tid] : 0;
    }
    if (tid == 0) flags[1] = 0;
    __syncthreads();
    const long long tmo = a.timeout_ticks;
    // ---- XCD discovery (as the batch-1 kernel): exactly 32 workgroups per XCD
    int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7;
    const unsigned setup_tag = (a.salt << 14) | 0x3FFFu;
    if (tid == 0) publish(a.gran + RBG_SETUP + c, setup_tag, __int_as_float(xcc));
    if (wave == 0) {
        float v4[4];
        const bool ok = sweep<4>(a.gran, setup_tag, v4, [&](int i) { return RBG_SETUP + lane * 4 + i; }, tmo);
        int rank = 0, nx = 0, nmin = RES_CUS, nmax = 0;
        const int xref = __builtin_amdgcn_readfirstlane(__float_as_int(v4[0]) & 7);
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
        if (nmax > RES_MIN_CUS_PER_XCD) nmin = 0;  // context channels 16 rank .. need exactly 32
        if (lane == 0) {
            flags[2] = rank;
            flags[3] = nx;
            flags[4] = xref;
            if (!ok) { flags[1] = 1; fail(a.status, 6); }
            else if (nmin < RES_MIN_CUS_PER_XCD) { flags[1] = 1; fail(a.status, RES_STATUS_PLACEMENT); }
        }
    }
    __syncthreads();
    if (flags[1]) return;
    const int rank = flags[2];
    const bool xlog = xcc == flags[4];  // the XCD whose copies write the outputs
    const bool stop_cu = rank == 0;
    // this wave's prenet-2 / prenet-1 rows of the XCD's copies (8 per CU, 2 per wave) and query row
    // (the query row's weights stay in registers; the prenet-1 rows' are fetched from the XCD's L2
    // each step while the h_dec hand-off is in flight)
    const int r0 = 8 * rank + 2 * wave;
    const float4 wp0 = ld4(a.w2 + r0 * PRE + lane * 4), wp1 = ld4(a.w2 + (r0 + 1) * PRE + lane * 4);
    const float bp1a = a.bf[a.nmel + r0], bp1b = a.bf[a.nmel + r0 + 1], bp2a = a.b2[r0], bp2b = a.b2[r0 + 1];
    const int qrow = 4 * rank + wave;
    const float* wql = sm + S::WQ + wave * HATT + lane * 4;
    for (int i = 0; i < 4; ++i) *reinterpret_cast<float4*>(sm + S::WQ + wave * HATT + i * 256 + lane * 4) = ld4(a.wq + qrow * HATT + i * 256 + lane * 4);
    const float* w1a = a.wf + (size_t)(a.nmel + r0) * KF + lane * 4;
    if (stop_cu && wave == 3)
        for (int i = 0; i < 6; ++i)
            reinterpret_cast<float4*>(rm)[(6 + i) * 64 + lane] = ld4(a.wf + (size_t)(a.nmel + PRE) * KF + i * 256 + lane * 4);
    const float stop_b = a.bf[a.nmel + PRE], mel_b = c < a.nmel ? a.bf[c] : 0.f;
    // the attention of sentence ab = wave (every CU of the XCD): this lane's dims 2 lane, 2 lane + 1
    const int ab = wave;
    const bool att_w = ab < NB;
    const int Lb = att_w ? a.L[ab] : 0;
    const int gf = a.gen;
    float gu = 0.5f, vb = 0.f;
    float2 gv = float2{0.f, 0.f};
    int gn = 1;
    if (att_w && Lb > 0) {
        gu = a.u[ab];
        gn = a.nidx[ab];
        vb = a.v_b[0];
        gv = *reinterpret_cast<const float2*>(a.v + 2 * lane);
        for (int k = lane; k < GW_PAD; k += 64) {
            const int j = k - 16;
            gw[(ab * 2) * GW_PAD + k] = j >= 0 && j < Lb ? a.alpha[(size_t)ab * a.Lcap + j] : 0.f;
            gw[(ab * 2 + 1) * GW_PAD + k] = 0.f;
        }
        // the CU's 16 context channels of sentence ab at every position, [j][16] (read each step)
        float* es = sm + S::ENCS + ab * S::ENC_L * 16;
        const float* src = a.enc + (size_t)ab * a.Lcap * ENC + 16 * rank;
        for (int k = lane; k < min(Lb, S::ENC_L) * 16; k += 64) es[k] = src[(size_t)(k >> 4) * ENC + (k & 15)];
    } else if (att_w) {
        for (int k = lane; k < 2 * GW_PAD; k += 64) gw[ab * 2 * GW_PAD + k] = 0.f;
    }
    // P of sentence ab (read each step from L2, issued before the query wait)
    const auto rpt = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.Pt + (size_t)(att_w ? ab : 0) * ADIM * a.Lcap),
                                                       (short)0, ADIM * a.Lcap * 4, 0x00020000);
    // this lane's P at the wave's positions rank + 32 i (dims 2 lane, 2 lane + 1): constant over the
    // launch, held in registers (a per-step reload held the query poll up behind ~1000 scattered
    // cache-line reads per wave: vmcnt is in order)
    float2 gp[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int pe = rank + 32 * i;
        const bool on = att_w && pe < Lb;
        gp[i].x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rpt, on ? (2 * lane * a.Lcap + pe) * 4 : OOB_OFF, 0, 0));
        gp[i].y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rpt, on ? ((2 * lane + 1) * a.Lcap + pe) * 4 : OOB_OFF, 0, 0));
    }
    const auto rg = __builtin_amdgcn_make_buffer_rsrc(a.gran, (short)0, 2 * RBG_TOTAL * 8, 0x00020000);
    const int xb = RBG_X + xcc * RBX_SIZE;  // this XCD's block (the parity offset is added per step)
    __syncthreads();
    if constexpr (PROF) tprev = (long long)wall_clock64();

    for (;; ++t) {
        const int P = (t & 1) * RBG_TOTAL, Pp = ((t & 1) ^ 1) * RBG_TOTAL;
        u64* G = a.gran + P;
        const unsigned E = (a.salt << 14) | (((unsigned)t & 2047u) << 3);
        const unsigned EP6 = ((a.salt << 14) | (((unsigned)(t - 1) & 2047u) << 3)) + 6u;
        // 1) attention LSTM over [ctx_{t-1} | h_att_{t-1}] for every sentence (acc[4 b + gate]); lane l
        //    reads k = 256 q + 4 l .. + 3 of each part (consecutive lanes, consecutive LDS banks)
        float acc[V];
#pragma unroll
        for (int i = 0; i < V; ++i) acc[i] = 0.f;
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            float* ac = acc + 4 * b;
#pragma unroll
            for (int q = 0; q < 2; ++q) fma44(wa + 4 + 4 * q, ld4(xctx + b * ENC + 256 * q + 4 * lane), ac);
#pragma unroll
            for (int q = 0; q < 4; ++q) fma44(wa + 12 + 4 * q, ld4(xh_att + b * HATT + 256 * q + 4 * lane), ac);
            asm volatile("" ::: "memory");  // one sentence's LDS operands in flight at a time
        }
        // the partial sums are computed HERE, off the critical path (while pre1 is in flight); without
        // the fence the compiler sinks these FMAs past the barriers into phase 4
#pragma unroll
        for (int i = 0; i < V; ++i) asm volatile("" : "+v"(acc[i]));
        mark(0);
        // 2) pre1_t (+ continue flags) of this XCD's copy, gathered from the previous step's parity
        if (t == 0) {
            for (int k = tid; k < NB * PRE; k += RB_THREADS) xp1[k] = k < a.B * PRE ? a.pre1[k] : 0.f;
        } else {
            const bool ok = gather_pairs<NB * PRE / 2>(rg, Pp + xb + RBX_P1, EP6, xp1, tmo);
            if (!ok && lane == 0) { flags[1] = 1; fail(a.status, 1, t); }
            if (wave == 0) {
                float f0 = 0.f, f1 = 0.f;
                const bool ok2 = sweep_pair(rg, lane < NB / 2 ? Pp + xb + RBX_FLAG + 2 * lane : -1, true, EP6, f0, f1, tmo);
                if (lane < NB / 2) {
                    act[2 * lane] = f0 != 0.f;
                    act[2 * lane + 1] = f1 != 0.f;
                }
                if (!ok2 && lane == 0) { flags[1] = 1; fail(a.status, 1, t); }
            }
        }
        __syncthreads();  // P1
        if (flags[1]) break;
        // the sentences decoding this step, as a register mask: wave 0 rewrites act[] for the next
        // step while other waves may still be in this step's last phase
        unsigned actm = 0;
#pragma unroll
        for (int b = 0; b < NB; ++b) actm |= act[b] ? 1u << b : 0u;
        if (!actm) break;
        mark(1);
        // 3) prenet layer 2: this wave's two rows of the XCD copy for every sentence (2 NB sums
        //    reduced together), XCD-local
        {
            float pv[2 * NB];
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const float4 x = ld4(xp1 + b * PRE + lane * 4);
                pv[2 * b] = dot4(wp0, x, 0.f);
                pv[2 * b + 1] = dot4(wp1, x, 0.f);
            }
            const float r = xreduce<2 * NB>(pv);
            constexpr int SP = 64 / (2 * NB);
            if ((lane & (SP - 1)) == 0) {
                const int idx = lane / SP, b = idx >> 1, rr = idx & 1;
                publish_xcd(G + xb + RBX_PRE2 + b * PRE + r0 + rr, E + 1, fmaxf(r + (rr ? bp2b : bp2a), 0.f));
            }
        }
        mark(2);
        {
            const bool ok = gather_pairs<NB * PRE / 2>(rg, P + xb + RBX_PRE2, E + 1, xpre, tmo, a.sleep_pre2);
            if (!ok && lane == 0) { flags[1] = 1; fail(a.status, 7, t); }
        }
        __syncthreads();  // P2
        if (flags[1]) break;
        mark(3);
        // 4) prenet part of the attention LSTM, reduction and cell of unit 4c + wave (this wave):
        //    publish h_att (device-wide)
#pragma unroll
        for (int b = 0; b < NB; ++b) fma44(wa, ld4(xpre + b * PRE + 4 * lane), acc + 4 * b);
        {
            const float r = xreduce<V>(acc);
            if ((lane & (64 / V - 1)) == 0) gsum[lane / (64 / V)] = r;
            // (the cell lanes read this wave's own LDS writes: in order, no barrier)
            if (cell_l) {
                const float4 z = ld4(gsum + 4 * lane);
                const float ig = sigmoid_cell(z.x + bia[0]), fg = sigmoid_cell(z.y + bia[1]);
                const float gg = tanh_cell(z.z + bia[2]), og = sigmoid_cell(z.w + bia[3]);
                c_att = fg * c_att + ig * gg;
                h_att_l = og * tanh_cell(c_att);
                publish(G + RBG_HATT + lane * HATT + 4 * c + wave, E + 2, h_att_l);
            }
        }
        // the decoder LSTM's h_dec_{t-1} half now: useful work before the first h_att poll (a poll
        // storm from every CU slows the hand-off it waits for)
        float accd[V];
#pragma unroll
        for (int i = 0; i < V; ++i) accd[i] = 0.f;
#pragma unroll
        for (int b = 0; b < NB; ++b) {
#pragma unroll
            for (int q = 0; q < 4; ++q) fma44(wd + 24 + 4 * q, ld4(xh_dec + b * HDEC + 256 * q + 4 * lane), accd + 4 * b);
            asm volatile("" ::: "memory");
        }
#pragma unroll
        for (int i = 0; i < V; ++i) asm volatile("" : "+v"(accd[i]));
        mark(4);
        // 5) gather h_att_t
        {
            const bool ok = gather_pairs<NB * HATT / 2>(rg, P + RBG_HATT, E + 2, xh_att, tmo, a.sleep_hatt);
            if (!ok && lane == 0) { flags[1] = 1; fail(a.status, 2, t); }
        }
        __syncthreads();  // P3
        if (flags[1]) break;
        mark(5);
        // 6) query row 4 rank + wave of the XCD copy for every sentence (common_layers.py:179), XCD-local
        {
            float qv[NB];
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                qv[b] = 0.f;
#pragma unroll
                for (int i = 0; i < 4; ++i) qv[b] = dot4(ld4(wql + i * 256), ld4(xh_att + b * HATT + i * 256 + lane * 4), qv[b]);
            }
            const float r = xreduce<NB>(qv);
            constexpr int SQ = 64 / NB;
            if ((lane & (SQ - 1)) == 0) publish_xcd(G + xb + RBX_Q + (lane / SQ) * ADIM + qrow, E + 3, r);
        }
        mark(6);
        // 7) attention of sentence ab in wave ab (common_layers.py:166-256 without location / windowing /
        //    transition agent), the context of this CU's 16 channels, XCD-local publish
        if (att_w && Lb == 0) {  // a padding sentence: zero context (every CU's gather waits for it)
            if (lane < 16) publish_xcd(G + xb + RBX_CTX + ab * ENC + 16 * rank + lane, E + 4, 0.f);
            if (rank == 0 && lane == 16) publish_xcd(G + xb + RBX_TAIL + ab, E + 4, 0.f);
        } else if (att_w) {
            float2 q = float2{0.f, 0.f};
            {
                const bool ok = sweep_pair(rg, P + xb + RBX_Q + ab * ADIM + 2 * lane, true, E + 3, q.x, q.y, tmo);
                if (!ok && lane == 0) { flags[1] = 1; fail(a.status, 3, t); }
            }
            mark(20);
            // the energy of positions rank + 32 i: v . tanh(q + P) + b_v (common_layers.py:178-182)
            {
                float ev[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) ev[i] = gv.x * tanh_fast(q.x + gp[i].x) + gv.y * tanh_fast(q.y + gp[i].y);
                const float r = xreduce<8>(ev);  // lane 8 i: position rank + 32 i
                const int pe = rank + 32 * (lane >> 3);
                if ((lane & 7) == 0 && pe < Lb) publish_xcd(G + xb + RBX_E + ab * RES_LMAX + pe, E + 7, r + vb);
            }
            mark(21);
            // sentence ab's energies from every CU of the XCD: positions 2 lane (+1), 128 + 2 lane (+1)
            int ps[4];
            bool in[4];
            float e[4];
            {
                const int eb = P + xb + RBX_E + ab * RES_LMAX;
                float e0 = 0.f, e1 = 0.f, e2 = 0.f, e3 = 0.f;
                bool ok = sweep_pair(rg, 2 * lane < Lb ? eb + 2 * lane : -1, 2 * lane + 1 < Lb, E + 7, e0, e1, tmo);
                ok = ok && sweep_pair(rg, 128 + 2 * lane < Lb ? eb + 128 + 2 * lane : -1, 129 + 2 * lane < Lb, E + 7, e2,
                                      e3, tmo);
                e[0] = e0; e[1] = e1; e[2] = e2; e[3] = e3;
                if (!ok && lane == 0) { flags[1] = 1; fail(a.status, 8, t); }
            }
            mark(22);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                ps[i] = (i >> 1) * 128 + 2 * lane + (i & 1);
                in[i] = ps[i] < Lb;
                if (!in[i]) e[i] = -INFINITY;
            }
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
                const float S_ = wave_sum_dpp((al[0] + al[1]) + (al[2] + al[3]));
#pragma unroll
                for (int i = 0; i < 4; ++i) al[i] = al[i] / S_;
            }
            const float* wold = gw + (ab * 2 + (t & 1)) * GW_PAD + 16;
            float* wnew = gw + (ab * 2 + ((t & 1) ^ 1)) * GW_PAD + 16;
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
                    const int cx = gn >= 2 ? gn - 2 : gn - 2 + Lb, lo = gn >= 1 ? gn - 1 : Lb - 1;
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
                        if (ps[i] <= Lb - 2 && w[i] > bv) { bv = w[i]; bi = ps[i]; }
                    wave_argmax(bv, bi);
                    gn = __builtin_amdgcn_readfirstlane(bv > 0.f ? bi + 1 : 0);
                }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) w[i] = al[i];
            }
            const float tail = wave_sum_dpp(((ps[0] >= Lb - 2 && in[0] ? w[0] : 0.f) + (ps[1] >= Lb - 2 && in[1] ? w[1] : 0.f)) +
                                            ((ps[2] >= Lb - 2 && in[2] ? w[2] : 0.f) + (ps[3] >= Lb - 2 && in[3] ? w[3] : 0.f)));
            *reinterpret_cast<float2*>(wnew + 2 * lane) = float2{w[0], w[1]};
            *reinterpret_cast<float2*>(wnew + 128 + 2 * lane) = float2{w[2], w[3]};
            mark(23);
            // the context of channels 16 rank + (lane & 15) over positions (lane >> 4) + 4 m (bmm, :217 /
            // :253) from the LDS copy; the weights were just written by this wave (in order)
            const float* es = sm + S::ENCS + ab * S::ENC_L * 16 + (lane & 15);
            float cacc = 0.f;
            int j = lane >> 4;
#pragma unroll 4
            for (; j < min(Lb, S::ENC_L); j += 4) cacc = fmaf(wnew[j], es[j * 16], cacc);
            if (Lb > S::ENC_L) {  // positions past the LDS copy (NB = 4, L > 128): from L2
                const float* encb = a.enc + (size_t)ab * a.Lcap * ENC + 16 * rank + (lane & 15);
                for (; j < Lb; j += 4) cacc = fmaf(wnew[j], encb[(size_t)j * ENC], cacc);
            }
            cacc = xlevel<16>(cacc, cacc);
            cacc = xlevel<32>(cacc, cacc);
            if (lane < 16) publish_xcd(G + xb + RBX_CTX + ab * ENC + 16 * rank + lane, E + 4, cacc);
            if (rank == 0 && lane == 16) publish_xcd(G + xb + RBX_TAIL + ab, E + 4, tail);
            if (xlog && rank == 0 && (actm >> ab & 1u) && t < a.hist_cap) {
                float* arow = a.align_hist + ((size_t)ab * a.hist_cap + t) * a.Lalign;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (ps[i] < a.Lalign) arow[ps[i]] = w[i];
            }
        }
        mark(7);
        // 8) decoder LSTM over [h_att_t | h_dec_{t-1}] (its partial sums are not held across the
        //    attention), while the other CUs' contexts arrive
#pragma unroll
        for (int i = 0; i < V; ++i) acc[i] = accd[i];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            float* ac = acc + 4 * b;
#pragma unroll
            for (int q = 0; q < 4; ++q) fma44(wd + 4 * q, ld4(xh_att + b * HATT + 256 * q + 4 * lane), ac);
            asm volatile("" ::: "memory");
        }
#pragma unroll
        for (int i = 0; i < V; ++i) asm volatile("" : "+v"(acc[i]));  // (as in phase 1: computed before the wait)
        mark(8);
        // 9) gather the NB contexts and tails
        {
            const bool ok = gather_pairs<NB * ENC / 2>(rg, P + xb + RBX_CTX, E + 4, xctx, tmo, a.sleep_ctx);
            if (!ok && lane == 0) { flags[1] = 1; fail(a.status, 4, t); }
            if (wave == 1) {
                float t0 = 0.f, t1 = 0.f;
                const bool ok2 = sweep_pair(rg, lane < NB / 2 ? P + xb + RBX_TAIL + 2 * lane : -1, true, E + 4, t0, t1, tmo);
                if (lane < NB / 2) {
                    xtail[2 * lane] = t0;
                    xtail[2 * lane + 1] = t1;
                }
                if (!ok2 && lane == 0) { flags[1] = 1; fail(a.status, 4, t); }
            }
        }
        __syncthreads();  // P4
        if (flags[1]) break;
        mark(9);
        // 10) decoder LSTM context part, reduction, cell -> publish h_dec (device-wide); this wave's
        //     prenet-1 row weights of step 12 are fetched meanwhile
        float4 wdc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) wdc[j] = reinterpret_cast<const float4*>(sm + S::WDC)[j * RB_THREADS + tid];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
#pragma unroll
            for (int q = 0; q < 2; ++q) fma44(wdc + 4 * q, ld4(xctx + b * ENC + 256 * q + 4 * lane), acc + 4 * b);
        }
        {
            const float r = xreduce<V>(acc);
            if ((lane & (64 / V - 1)) == 0) gsum[lane / (64 / V)] = r;
            if (cell_l) {
                const float4 z = ld4(gsum + 4 * lane);
                const float ig = sigmoid_cell(z.x + bid[0]), fg = sigmoid_cell(z.y + bid[1]);
                const float gg = tanh_cell(z.z + bid[2]), og = sigmoid_cell(z.w + bid[3]);
                c_dec = fg * c_dec + ig * gg;
                h_dec_l = og * tanh_cell(c_dec);
                publish(G + RBG_HDEC + lane * HDEC + 4 * c + wave, E + 5, h_dec_l);
            }
        }
        mark(10);
        // 11) gather h_dec_t (this wave's prenet-1 row weights of step 12 in flight meanwhile)
        float4 w1p[12];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            w1p[i] = ld4(w1a + i * 256);
            w1p[6 + i] = ld4(w1a + KF + i * 256);
        }
        {
            const bool ok = gather_pairs<NB * HDEC / 2>(rg, P + RBG_HDEC, E + 5, xh_dec, tmo, a.sleep_hdec);
            if (!ok && lane == 0) { flags[1] = 1; fail(a.status, 5, t); }
        }
        __syncthreads();  // P5
        if (flags[1]) break;
        mark(11);
        // 12) prenet-1 rows of step t+1 (XCD copy) over [h_dec_t | ctx_t], XCD-local; the stop CU's
        //     wave 3: stopnet + stop rule per sentence -> continue flags; CU c < nmel: mel row c
        {
            float pv[2 * NB];
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                float s0 = 0.f, s1 = 0.f;
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    const float4 x = i < 4 ? ld4(xh_dec + b * HDEC + i * 256 + lane * 4) : ld4(xctx + b * ENC + (i - 4) * 256 + lane * 4);
                    s0 = dot4(w1p[i], x, s0);
                    s1 = dot4(w1p[6 + i], x, s1);
                }
                pv[2 * b] = s0;
                pv[2 * b + 1] = s1;
            }
            const float r = xreduce<2 * NB>(pv);
            constexpr int SP = 64 / (2 * NB);
            if ((lane & (SP - 1)) == 0) {
                const int idx = lane / SP, b = idx >> 1, rr = idx & 1;
                publish_xcd(G + xb + RBX_P1 + b * PRE + r0 + rr, E + 6, fmaxf(r + (rr ? bp1b : bp1a), 0.f));
            }
        }
        if ((stop_cu && wave == 3) || (wave == 1 && c < a.nmel)) {
            // stop CU wave 3: the stopnet row; wave 1 of CU c < nmel: mel row c (LDS copies)
            const float4* wr = reinterpret_cast<const float4*>(rm) + (wave == 3 ? 6 * 64 : 0) + lane;
            float sv[NB];
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                float s = 0.f;
#pragma unroll
                for (int i = 0; i < 4; ++i) s = dot4(wr[i * 64], ld4(xh_dec + b * HDEC + i * 256 + lane * 4), s);
#pragma unroll
                for (int i = 4; i < 6; ++i) s = dot4(wr[i * 64], ld4(xctx + b * ENC + (i - 4) * 256 + lane * 4), s);
                sv[b] = s;
            }
            const float ss = xreduce<NB>(sv);
            constexpr int SQ = 64 / NB;
            const int b = lane / SQ;  // lanes SQ b: sentence b
            const bool actb = (actm >> b & 1u) != 0;
            if ((lane & (SQ - 1)) == 0 && wave == 1) {
                if (actb && t < a.hist_cap) a.mel_hist[((size_t)b * a.hist_cap + t) * a.nmel + c] = ss + mel_b;
            } else if ((lane & (SQ - 1)) == 0) {
                // stopnet + stop rule (tacotron2.py:219-224, 257-277) of sentence b, as a batch-1 run
                int cont = 0;
                if (actb) {
                    const float stv = sigmoidf_(ss + stop_b);
                    if (xlog && t < a.hist_cap) a.stop_hist[(size_t)b * a.hist_cap + t] = stv;
                    int Lsb = a.L[0];
#pragma unroll
                    for (int k = 1; k < NB; ++k)
                        if (b == k) Lsb = a.L[k];
                    const int f1 = sflag1[b] | ((xtail[b] > 0.8f && t > Lsb) ? 1 : 0);
                    sflag1[b] = f1;
                    int nd = 0;
                    if (f1 && t > 2 * Lsb) {
                        scount[b] += 1;
                        if (scount[b] > 20) nd = 1;
                    } else if (t + 1 == a.max_steps) {
                        nd = 1;
                    }
                    if (!nd && t + 1 >= a.hist_cap) {  // cannot happen: the rule stops by max_steps + 20
                        nd = 1;
                        fail(a.status, 100);
                    }
                    if (nd && xlog) {
                        a.done[b] = 1;
                        a.n_steps[b] = t + 1;
                    }
                    cont = !nd;
                }
                publish_xcd(G + xb + RBX_FLAG + b, E + 6, cont ? 1.f : 0.f);
            }
        }
        mark(12);
    }
    if constexpr (PROF) {
        if (lane == 0) {
            long long* pr = a.prof + (size_t)(c * 4 + wave) * RB_PROF_SLOTS;
#pragma unroll
            for (int k = 0; k < RB_PROF_SLOTS - 1; ++k) pr[k] = ptk[k];
            pr[RB_PROF_SLOTS - 1] = t;
        }
    }
    if (flags[1]) return;
    // the last step t-1 leaves its state where the multi-launch path's would be
    const int pl = (t - 1) & 1;
    if (cell_l && lane < a.B) {
        a.h_att[pl * a.hps + (size_t)lane * HATT + 4 * c + wave] = h_att_l;
        a.c_att[(size_t)lane * HATT + 4 * c + wave] = c_att;
        a.h_dec[pl * a.hps + (size_t)lane * HDEC + 4 * c + wave] = h_dec_l;
        a.c_dec[(size_t)lane * HDEC + 4 * c + wave] = c_dec;
    }
}

// ---- weight packing (once, at tts_decoder_create): CU c, wave (= unit) u, lane (= k-slice) l,
// register j: float4 of the 4 gates (torch order i, f, g, o) at one k
__global__ void rb_pack_wa(const float* wih, const float* whh, float4* out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)RES_CUS * KA * RB_THREADS) return;
    const int tid = idx % RB_THREADS, j = (idx / RB_THREADS) % KA, c = idx / (KA * RB_THREADS);
    const int uu = tid >> 6, l = tid & 63;
    // k over [prenet 256 | ctx 512 | h_att 1024]: 4 + 8 + 16 per lane, k = 256 q + 4 l + e in each part
    const int jj = j < 4 ? j : j < 12 ? j - 4 : j - 12;
    const int k = (j < 4 ? 0 : j < 12 ? PRE : XA) + 256 * (jj >> 2) + 4 * l + (jj & 3);
    float v[4];
    for (int g = 0; g < 4; ++g) {
        const int row = g * HATT + 4 * c + uu;
        v[g] = k < XA ? wih[(int64_t)row * XA + k] : whh[(int64_t)row * HATT + (k - XA)];
    }
    out[idx] = float4{v[0], v[1], v[2], v[3]};
}
__global__ void rb_pack_wd(const float* wih, const float* whh, float4* out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)RES_CUS * KD * RB_THREADS) return;
    const int tid = idx % RB_THREADS, j = (idx / RB_THREADS) % KD, c = idx / (KD * RB_THREADS);
    const int uu = tid >> 6, l = tid & 63;
    // k over [h_att 1024 | ctx 512 | h_dec 1024]: 16 + 8 + 16 per lane, k = 256 q + 4 l + e in each part
    const int jj = j < 16 ? j : j < 24 ? j - 16 : j - 24;
    const int k = (j < 16 ? 0 : j < 24 ? HATT : HATT + ENC) + 256 * (jj >> 2) + 4 * l + (jj & 3);
    float v[4];
    for (int g = 0; g < 4; ++g) {
        const int row = g * HDEC + 4 * c + uu;
        v[g] = k < HATT + ENC ? wih[(int64_t)row * (HATT + ENC) + k] : whh[(int64_t)row * HDEC + (k - HATT - ENC)];
    }
    out[idx] = float4{v[0], v[1], v[2], v[3]};
}

int rb_nb(int B) { return B <= 2 ? 2 : 4; }

}  // namespace

void resident_batch_weight_floats(size_t* wa, size_t* wd) {
    *wa = (size_t)RES_CUS * KA * RB_THREADS * 4;
    *wd = (size_t)RES_CUS * KD * RB_THREADS * 4;
}

size_t resident_batch_granules() { return 2 * (size_t)RBG_TOTAL; }

hipError_t resident_batch_pack(const ResSrc& s, float4* wa, float4* wd, hipStream_t st) {
    auto blocks = [](int64_t n) { return dim3((unsigned)((n + 255) / 256)); };
    hipLaunchKernelGGL(rb_pack_wa, blocks((int64_t)RES_CUS * KA * RB_THREADS), dim3(256), 0, st, s.a_wih, s.a_whh, wa);
    hipLaunchKernelGGL(rb_pack_wd, blocks((int64_t)RES_CUS * KD * RB_THREADS), dim3(256), 0, st, s.d_wih, s.d_whh, wd);
    return hipGetLastError();
}

size_t resident_batch_smem_bytes(int B) {
    return (size_t)(rb_nb(B) == 2 ? Lds<2>::TOTAL : Lds<4>::TOTAL) * sizeof(float);
}

hipError_t resident_batch_prepare() {
    const void* fns[] = {reinterpret_cast<const void*>(&resident_batch_kernel<2, false>),
                         reinterpret_cast<const void*>(&resident_batch_kernel<4, false>),
                         reinterpret_cast<const void*>(&resident_batch_kernel<2, true>),
                         reinterpret_cast<const void*>(&resident_batch_kernel<4, true>)};
    const int nbs[] = {2, 4, 2, 4};
    for (int i = 0; i < 4; ++i) {
        hipError_t e = hipFuncSetAttribute(fns[i], hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)resident_batch_smem_bytes(nbs[i]));
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

bool resident_batch_supports(int gen) { return gen != 0 && !(gen & (GEN_TA | GEN_LOCATION | GEN_WINDOW)); }

hipError_t launch_resident_batch(const ResBatchArgs& a, hipStream_t s, bool* launched) {
    *launched = false;
    if (a.B < 1 || a.B > RB_MAXB || a.nmel > RES_CUS || a.nmel + PRE + 1 != a.nrows || !resident_batch_supports(a.gen))
        return hipErrorInvalidValue;
    for (int b = 0; b < a.B; ++b)
        if (a.L[b] < 2 || a.L[b] > RES_LMAX || a.L[b] > a.Lcap) return hipErrorInvalidValue;
    ResBatchArgs arg = a;
    for (int b = a.B; b < RB_MAXB; ++b) arg.L[b] = 0;
    void* args[] = {&arg};
    const bool prof = a.prof != nullptr;
    const void* fn = rb_nb(a.B) == 2 ? (prof ? reinterpret_cast<const void*>(&resident_batch_kernel<2, true>)
                                             : reinterpret_cast<const void*>(&resident_batch_kernel<2, false>))
                                     : (prof ? reinterpret_cast<const void*>(&resident_batch_kernel<4, true>)
                                             : reinterpret_cast<const void*>(&resident_batch_kernel<4, false>));
    return launch_persistent(fn, dim3(RES_CUS), dim3(RB_THREADS), args, resident_batch_smem_bytes(a.B), s, launched);
}

}  // namespace tts

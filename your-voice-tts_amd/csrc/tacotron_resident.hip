// Resident TacotronGST / Tacotron decoder: the whole Decoder.inference loop (layers/tacotron.py:
// 439-470, decode :366-394) in ONE persistent launch of 256 workgroups (one per CU, 512 threads).
//
// XCD groups.  The step weights are 6.7 MB: every XCD holds a full copy on its 32 CUs (106 VGPRs
// per thread) and runs its own group of up to TR_SPX = 4 sentences (sentence b on the XCD with
// id b / 4), so no hand-off ever leaves an XCD: each is an 8-byte {tag, value} granule stored
// workgroup-scope (the line stays in the XCD's L2) and polled with sc1 loads, as in the batch-1
// Tacotron2 resident decoder (resident_decoder.hip).
//
// Step t of a group, CU rank r (0..31), wave w, one hand-off per arrow (all four sentences at once):
//   pre1 -> [prenet L2: waves 0-3, rows 4r + w]
//        -> [attention GRU: unit 8r + w over [prenet | ctx_{t-1}] and h_att_{t-1}]
//        -> [query_layer: waves 4-7, rows 4r + w - 4]
//        -> [attention: the 8 CUs of sentence r / 8 each own 32 encoder positions (P and the encoder
//            rows staged in LDS at launch): energies, sigmoid, forward-attention weights
//            w_j = ((1-u) a_j + u a_{j-1} + 1e-8) sig(e_j) and the partial sums sum w, sum w enc]
//        -> [the sentence's first CU adds the 8 partials in slice order: ctx, the normaliser,
//            alpha at the slice boundaries and at L-1]
//        -> [project_to_decoder_in: row 8r + w] -> [decoder GRU 1 + residual] -> [GRU 2 + residual]
//        -> [proj_to_mel + sigmoid: rows r + 32 w, r + 32 (w + 8); mel history]
//        -> [prenet L1 of t+1: row 8r + w; rank 0: stopnet over [decoder out | mel] + stop rule]
// The forward-attention normalisation uses alpha = w / sum(w): the sigmoid normaliser of the
// reference (alignment = sig / sum sig) cancels in it, so it is not reduced (same values up to
// float32 rounding).  Every other reduction follows a fixed order (bitwise run-to-run
// deterministic).  Every wait is bounded; a timed-out wait flags the status and drains the grid.
#include "tacotron.h"

namespace tts {
namespace {

typedef unsigned long long u64;
typedef __attribute__((address_space(1))) u64 gu64;
typedef __attribute__((address_space(1))) int gint;

constexpr int TD = T_DEC;                    // 256
constexpr int ADIM = 128;                    // attention_dim
constexpr int TXA = T_PRE2 + T_DEC;          // attention-GRU input [prenet 128 | ctx 256]
constexpr int ATTP_W = TD + 4;               // attention partial: sum w enc [256], sum w, w_last, w_{L-1}
constexpr int CTXF_W = TD + 2 + TR_CPS + 6;  // ctx [256], normaliser, tail, alpha at slice ends [8]
// granule offsets inside one group's block (one block per group and step parity)
constexpr int G_PRE2 = 0;
constexpr int G_HATT = G_PRE2 + TR_SPX * T_PRE2;
constexpr int G_Q = G_HATT + TR_SPX * TD;
constexpr int G_ATTP = G_Q + TR_SPX * ADIM;
constexpr int G_CTXF = G_ATTP + TR_SPX * TR_CPS * ATTP_W;
constexpr int G_DIN = G_CTXF + TR_SPX * CTXF_W;
constexpr int G_H1 = G_DIN + TR_SPX * TD;   // h1 [SPX][256] then d1 [SPX][256]
constexpr int G_H2 = G_H1 + 2 * TR_SPX * TD;
constexpr int G_MEL = G_H2 + 2 * TR_SPX * TD;
constexpr int G_PRE1 = G_MEL + TR_SPX * TR_NMEL_MAX;  // pre1 [SPX][256] then the continue flags [SPX]
constexpr int G_GROUP = G_PRE1 + TR_SPX * T_PRE1 + 16;
constexpr int G_PARITY = TR_GROUPS * G_GROUP;
constexpr int G_SETUP = 2 * G_PARITY;       // [256] XCD id of every CU
constexpr int G_TOTAL = G_SETUP + TR_CUS;
// phase ids (tag low bits)
enum { P_PRE2 = 1, P_HATT, P_Q, P_ATTP, P_CTXF, P_DIN, P_H1, P_H2, P_MEL, P_PRE1 };

// LDS layout (floats)
constexpr int L_XA = 0;                                  // [SPX][384] [prenet | ctx]
constexpr int L_HATT = L_XA + TR_SPX * TXA;              // [2][SPX][256] by step parity
constexpr int L_PRE1 = L_HATT + 2 * TR_SPX * TD;         // [SPX][256]
constexpr int L_DIN = L_PRE1 + TR_SPX * T_PRE1;          // [SPX][256]
constexpr int L_H1 = L_DIN + TR_SPX * TD;                // [2][SPX][256]
constexpr int L_D1 = L_H1 + 2 * TR_SPX * TD;             // [SPX][256]
constexpr int L_H2 = L_D1 + TR_SPX * TD;                 // [2][SPX][256]
constexpr int L_D2 = L_H2 + 2 * TR_SPX * TD;             // [SPX][256]
constexpr int L_MEL = L_D2 + TR_SPX * TD;                // [SPX][512]
constexpr int L_Q = L_MEL + TR_SPX * TR_NMEL_MAX;        // [128] this CU's attention sentence
constexpr int L_V = L_Q + ADIM;                          // [128]
constexpr int L_PS = L_V + ADIM;                         // [32][128] P of this CU's positions
constexpr int L_ES = L_PS + TR_PPC * ADIM;               // [32][256] encoder rows of them
constexpr int L_AL = L_ES + TR_PPC * TD;                 // [32] alpha of them, then [1] boundary alpha
constexpr int L_WJ = L_AL + TR_PPC + 16;                 // [32] this step's unnormalised weights
constexpr int L_RED = L_WJ + TR_PPC + 16;                // [2][280] partial / leader scratch
constexpr int L_STOP = L_RED + 2 * 280;                  // [256 + 512] stopnet row (rank 0)
constexpr int L_BIAS = L_STOP + TD + TR_NMEL_MAX;        // [8 waves][16] per-wave biases
constexpr int L_CTL = L_BIAS + TR_WAVES * 16;            // [SPX] normaliser, [SPX] tail, [SPX][8] bnd, ints
constexpr int L_W1 = L_CTL + TR_SPX * (2 + TR_CPS) + 32; // [8 waves][8][64] prenet-L1 row U (lane-strided)
constexpr int L_WM = L_W1 + TR_WAVES * 8 * 64;           // [8 waves][8][64] proj_to_mel rows m0 (0-3), m1 (4-7)
constexpr int L_PROF = L_WM + TR_WAVES * 8 * 64;          // [TR_PHASES] u64 phase timers (measurement)
constexpr int L_TOTAL = L_PROF + 2 * TR_PHASES;

__device__ __forceinline__ void publish(u64* g, unsigned tag, float v) {
    __hip_atomic_store((gu64*)g, ((u64)tag << 32) | (u64)__float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void publish_agent(u64* g, unsigned tag, float v) {
    __hip_atomic_store((gu64*)g, ((u64)tag << 32) | (u64)__float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 peek(u64* g) {
    return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void fail(int* status, int code) {
    __hip_atomic_store((gint*)status, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// One wave polls its N granules per lane (idx(i) < 0: none) until every tag equals `tag`; false
// after `tmo` wall-clock ticks.
template <int N, typename F>
__device__ __forceinline__ bool sweep(u64* g, unsigned tag, float (&v)[N], F idx, long long tmo, int first_sleep = 0) {
    long long t_end = 0;
    // (a poll storm from every CU of the XCD the moment it has published slows the stores it waits for)
    for (int i = 0; i < first_sleep; ++i) __builtin_amdgcn_s_sleep(1);
    for (int spin = 0;; ++spin) {
        bool ok = true;
        // every load issued unconditionally (a slot with idx < 0 re-reads slot 0 and is ignored), so
        // the N loads of a poll are in flight together
        u64 x[N];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const int k = idx(i);
            x[i] = peek(g + (k >= 0 ? k : 0));
        }
#pragma unroll
        for (int i = 0; i < N; ++i) {
            v[i] = __uint_as_float((unsigned)x[i]);
            ok = ok & ((idx(i) < 0) | ((unsigned)(x[i] >> 32) == tag));  // no short-circuit branches
        }
        if (__all(ok)) return true;
        if (spin == 0) {
            t_end = (long long)wall_clock64() + tmo;
        } else if ((spin & 31) == 1 && (long long)wall_clock64() > t_end) {
            return false;
        }
    }
}
// sum over the 16 lanes of each DPP row: the total lands in lane 15 of the row
__device__ __forceinline__ float row_sum16(float v) {
    v += dpp_move<0x111, 0xf>(v, 0.f);
    v += dpp_move<0x112, 0xf>(v, 0.f);
    v += dpp_move<0x114, 0xf>(v, 0.f);
    v += dpp_move<0x118, 0xf>(v, 0.f);
    return v;
}
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float2 ld2(const float* p) { return *reinterpret_cast<const float2*>(p); }
template <int CTRL>
__device__ __forceinline__ float dpp_all(float v) {  // full-wave DPP move, every lane written
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
// partner of `lane` at halving stage st (0..3): xor 32, xor 16, xor 8, mirror within 8 (xor 7);
// every pair differs in bit 5 - st, which picks the half a lane keeps
template <int ST>
__device__ __forceinline__ float partner(float v) {
    if constexpr (ST == 0) return __shfl_xor(v, 32, 64);
    else if constexpr (ST == 1) return __shfl_xor(v, 16, 64);
    else if constexpr (ST == 2) return dpp_all<0x128>(v);  // row_ror:8
    else return dpp_all<0x141>(v);                         // row_half_mirror
}
// Transposed wave reduction of N in {4, 8, 16} per-lane partial sums: log2(N) halving stages
// (each lane keeps half of its values, adding its partner's copy of them), then plain sums over
// the remaining lane bits.  The total of value k ends in lane (64 / N) k (and its neighbours
// (64 / N) k + 1..3); 2 N - 1 + (6 - log2 N) lane moves instead of 6 N.  Fixed order per value.
template <int N, int ST = 0>
__device__ __forceinline__ float xreduce(const float (&v)[N], int lane) {
    if constexpr (N == 1) {
        float x = v[0];
        if constexpr (ST <= 0) x += partner<0>(x);
        if constexpr (ST <= 1) x += partner<1>(x);
        if constexpr (ST <= 2) x += partner<2>(x);
        if constexpr (ST <= 3) x += partner<3>(x);
        x += dpp_all<0x4E>(x);  // quad_perm [2,3,0,1]
        x += dpp_all<0xB1>(x);  // quad_perm [1,0,3,2]
        return x;
    } else {
        const bool hi = (lane >> (5 - ST)) & 1;
        float w[N / 2];
#pragma unroll
        for (int k = 0; k < N / 2; ++k) {
            const float keep = hi ? v[k + N / 2] : v[k];
            const float send = hi ? v[k] : v[k + N / 2];
            w[k] = keep + partner<ST>(send);
        }
        return xreduce<N / 2, ST + 1>(w, lane);
    }
}
// p[s] = sum_i w[i] * x[s * ld + 4 lane + i] (i < 4) for the group's four sentences
__device__ __forceinline__ void dot4(float (&p)[TR_SPX], const float* w, const float* x, int ld, int lane) {
#pragma unroll
    for (int s = 0; s < TR_SPX; ++s) {
        const float4 xv = ld4(x + s * ld + 4 * lane);
        p[s] = fmaf(w[3], xv.w, fmaf(w[2], xv.z, fmaf(w[1], xv.y, w[0] * xv.x)));
    }
}
// totals of four sentences' partials, sentence s's total returned in lane s (lanes 0-3)
__device__ __forceinline__ float to_lanes(const float (&p)[TR_SPX], int lane) {
    const float tot = xreduce<TR_SPX>(p, lane);
    return __shfl(tot, 16 * (lane & 3), 64);
}

__global__ __launch_bounds__(TR_THREADS, 1) void tacotron_resident_kernel(const TResArgs a) {
    const int c = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    extern __shared__ __align__(16) float sm[];
    int* ctl = reinterpret_cast<int*>(sm + L_CTL + TR_SPX * (2 + TR_CPS));  // [0] abort, [1] rank, [2] nx, [3] all done, [4..8) done
    const long long tmo = a.timeout_ticks;
    const int fsl = a.first_sleep;
    // phase timers (measurement only, tts_tacotron_resident_phases): CUs 0 and 1 of group 0
    bool prof = false;
    long long plast = 0;
    unsigned long long* pacc = reinterpret_cast<unsigned long long*>(sm + L_PROF);
#define MARK(k)                                                 \
    if (prof && tid == 0) {                                     \
        const long long now_ = (long long)wall_clock64();       \
        pacc[k] += (unsigned long long)(now_ - plast);          \
        plast = now_;                                           \
    }
    // ---- XCD discovery: rank = #CUs of this XCD with a lower block index
    int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7;
    const unsigned setup_tag = (a.salt << 14) | 0x3FFFu;
    if (tid == 0) publish_agent(a.gran + G_SETUP + c, setup_tag, __int_as_float(xcc));
    if (tid == 0) ctl[0] = 0;
    if (wave == 0) {
        float v4[4];
        const bool ok = sweep<4>(a.gran + G_SETUP, setup_tag, v4, [&](int i) { return lane * 4 + i; }, tmo);
        int rank = 0, nx = 0, nmin = TR_CUS;
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
        }
        if (lane == 0) {
            ctl[1] = rank;
            ctl[2] = nx;
            if (!ok) { ctl[0] = 1; fail(a.status, 9); }
            else if (nmin < TR_RANKS) { ctl[0] = 1; fail(a.status, TR_STATUS_PLACEMENT); }
        }
    }
    __syncthreads();
    if (ctl[0]) return;
    const int r = ctl[1];
    prof = a.prof != nullptr && xcc == 0 && r < 2;
    if (prof && tid < TR_PHASES) pacc[tid] = 0;
    const int b0 = xcc * TR_SPX;                         // this group's first sentence
    const int ns = min(TR_SPX, a.B - b0);                // its sentences
    if (r >= TR_RANKS || ns <= 0) return;                // idle CU / group
    const int nmel = a.nmel;
    // ---- weights into registers (reference layouts): lane l holds k = 4l + i of every 256-wide
    // segment (one ds_read_b128 of the input per segment), k = 2l + i of the 128-wide prenet part
    const int U = 8 * r + wave;  // attention-GRU / decoder-GRU unit, proj row, prenet-L1 row
    float axr[6], axz[6], axn[6], ahr[4], ahz[4], ahn[4];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int k = i < 2 ? 2 * lane + i : T_PRE2 + 4 * lane + (i - 2);
        axr[i] = a.a_wih[(int64_t)U * TXA + k];
        axz[i] = a.a_wih[(int64_t)(TD + U) * TXA + k];
        axn[i] = a.a_wih[(int64_t)(2 * TD + U) * TXA + k];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = 4 * lane + i;
        ahr[i] = a.a_whh[(int64_t)U * TD + k];
        ahz[i] = a.a_whh[(int64_t)(TD + U) * TD + k];
        ahn[i] = a.a_whh[(int64_t)(2 * TD + U) * TD + k];
    }
    float gx[2][3][4], gh[2][3][4];
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                gx[g][q][i] = a.g_wih[g][(int64_t)(q * TD + U) * TD + 4 * lane + i];
                gh[g][q][i] = a.g_whh[g][(int64_t)(q * TD + U) * TD + 4 * lane + i];
            }
    float wp[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) wp[i] = a.w_proj[(int64_t)U * 2 * TD + (i < 4 ? 4 * lane + i : TD + 4 * lane + i - 4)];
    const int m0 = r + 32 * wave, m1 = r + 32 * (wave + 8);  // this wave's mel rows (if < nmel)
    // these two are read from LDS (register budget), one float4 per lane and segment:
    // wm [row m0 | row m1][lane][4] (k = 4 lane + i), w1 [2][lane][4] (k = 8 lane + 4 h + i)
    float* wm = sm + L_WM + wave * 8 * 64;
    float* w1 = sm + L_W1 + wave * 8 * 64;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        wm[lane * 4 + i] = m0 < nmel ? a.w_mel[(int64_t)m0 * TD + 4 * lane + i] : 0.f;
        wm[256 + lane * 4 + i] = m1 < nmel ? a.w_mel[(int64_t)m1 * TD + 4 * lane + i] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int k = 8 * lane + i;
        w1[(i >> 2) * 256 + lane * 4 + (i & 3)] = k < nmel ? a.w_pre1[(int64_t)U * nmel + k] : 0.f;
    }
    const int r2 = 4 * r + (wave & 3);  // prenet-L2 row (waves 0-3) / query row (waves 4-7)
    float w2q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        w2q[i] = wave < 4 ? a.w_pre2[(int64_t)r2 * TD + 4 * lane + i] : a.w_q[(int64_t)r2 * TD + 4 * lane + i];
    // per-wave biases (LDS): [0..3] attention GRU r, z, n_x, n_h; [4..11] decoder GRUs; [12] proj;
    // [13] prenet L1; [14] prenet L2 (waves 0-3); [15] unused; mel biases by row below
    float* bias = sm + L_BIAS + wave * 16;
    if (lane == 0) {
        bias[0] = a.a_bih[U] + a.a_bhh[U];
        bias[1] = a.a_bih[TD + U] + a.a_bhh[TD + U];
        bias[2] = a.a_bih[2 * TD + U];
        bias[3] = a.a_bhh[2 * TD + U];
        for (int g = 0; g < 2; ++g) {
            bias[4 + 4 * g] = a.g_bih[g][U] + a.g_bhh[g][U];
            bias[5 + 4 * g] = a.g_bih[g][TD + U] + a.g_bhh[g][TD + U];
            bias[6 + 4 * g] = a.g_bih[g][2 * TD + U];
            bias[7 + 4 * g] = a.g_bhh[g][2 * TD + U];
        }
        bias[12] = a.b_proj[U];
        bias[13] = a.b_pre1[U];
        bias[14] = wave < 4 ? a.b_pre2[r2] : 0.f;
    }
    const float bm0 = m0 < nmel ? a.b_mel[m0] : 0.f, bm1 = m1 < nmel ? a.b_mel[m1] : 0.f;
    // ---- attention slice: sentence sa = r / 8, positions [ka * 32, ka * 32 + 32)
    const int sa = r / TR_CPS, ka = r % TR_CPS;
    const bool att_on = sa < ns;
    const int ba = b0 + sa;
    const int La = att_on ? a.lens[ba] : 0;
    const int j0 = ka * TR_PPC;
    float* Ps = sm + L_PS;
    float* Es = sm + L_ES;
    float* al = sm + L_AL;
    float* wj = sm + L_WJ;
    if (att_on) {
        for (int i = tid; i < TR_PPC * ADIM; i += TR_THREADS) {
            const int jl = i / ADIM, d = i % ADIM, j = j0 + jl;
            Ps[i] = j < La ? a.Pt[((int64_t)ba * ADIM + d) * a.Lcap + j] : 0.f;
        }
        for (int i = tid; i < TR_PPC * TD; i += TR_THREADS) {
            const int jl = i / TD, d = i % TD, j = j0 + jl;
            Es[i] = j < La ? a.enc[((int64_t)ba * a.Lcap + j) * TD + d] : 0.f;
        }
        if (tid < TR_PPC) al[tid] = j0 + tid < a.Lcap ? a.alpha[(int64_t)ba * a.Lcap + j0 + tid] : 0.f;
        if (tid == TR_PPC) al[TR_PPC] = j0 > 0 ? a.alpha[(int64_t)ba * a.Lcap + j0 - 1] : 0.f;
    }
    if (tid < ADIM) sm[L_V + tid] = a.v[tid];
    const float vb = a.v_b[0];
    // stopnet row (rank 0): [decoder out 256 | mel nmel]
    if (r == 0)
        for (int k = tid; k < TD + TR_NMEL_MAX; k += TR_THREADS) sm[L_STOP + k] = k < TD + nmel ? a.w_stop[k] : 0.f;
    const float bstop = a.b_stop[0];
    // ---- initial state (slot 1 of h, context 0, prenet L1 of the go frame)
    for (int i = tid; i < TR_SPX * TD; i += TR_THREADS) {
        const int s = i / TD, k = i % TD, b = b0 + s;
        const bool on = s < ns;
        sm[L_HATT + TR_SPX * TD + i] = on ? a.h_att[a.h_pstride + (int64_t)b * TD + k] : 0.f;
        sm[L_H1 + TR_SPX * TD + i] = on ? a.h1[a.h_pstride + (int64_t)b * TD + k] : 0.f;
        sm[L_H2 + TR_SPX * TD + i] = on ? a.h2[a.h_pstride + (int64_t)b * TD + k] : 0.f;
        sm[L_PRE1 + i] = on ? a.pre1[(int64_t)b * T_PRE1 + k] : 0.f;
    }
    for (int i = tid; i < TR_SPX * TXA; i += TR_THREADS) sm[L_XA + i] = 0.f;
    for (int i = tid; i < TR_SPX * TR_NMEL_MAX; i += TR_THREADS) sm[L_MEL + i] = 0.f;
    int* dn = ctl + 4;  // done flags of the group's sentences (as of this step's start)
    if (tid < TR_SPX) dn[tid] = tid < ns ? 0 : 1;
    int Ls[TR_SPX];
#pragma unroll
    for (int s = 0; s < TR_SPX; ++s) Ls[s] = s < ns ? a.lens[b0 + s] : 0;
    float* nrm = sm + L_CTL;                 // [SPX] attention normaliser of this step
    float* tl = nrm + TR_SPX;                // [SPX] alpha[L-1]
    float* bnd = tl + TR_SPX;                // [SPX][8] alpha at the slice ends
    int st_flag1 = 0;
    (void)st_flag1;
    __syncthreads();

    float* xa = sm + L_XA;
    float* pre1 = sm + L_PRE1;
    float* din = sm + L_DIN;
    float* d1 = sm + L_D1;
    float* d2 = sm + L_D2;
    float* mel = sm + L_MEL;
    float* q = sm + L_Q;
    float* red = sm + L_RED;
    if (prof && tid == 0) plast = (long long)wall_clock64();
    for (int t = 0;; ++t) {
        // the lane index as an opaque per-step value: the hand-off indices below are recomputed
        // every step instead of being hoisted out of the loop as 64-bit offsets (register budget)
        int ln = lane;
        asm volatile("" : "+v"(ln));
        u64* G = a.gran + (t & 1) * G_PARITY + xcc * G_GROUP;
        u64* Gp = a.gran + ((t & 1) ^ 1) * G_PARITY + xcc * G_GROUP;
        const unsigned E = (a.salt << 14) | ((unsigned)(t & 1023) << 4);
        const unsigned Ep = (a.salt << 14) | ((unsigned)((t - 1) & 1023) << 4);
        float* hatt_prev = sm + L_HATT + ((t + 1) & 1) * TR_SPX * TD;
        float* hatt = sm + L_HATT + (t & 1) * TR_SPX * TD;
        float* h1_prev = sm + L_H1 + ((t + 1) & 1) * TR_SPX * TD;
        float* h1 = sm + L_H1 + (t & 1) * TR_SPX * TD;
        float* h2_prev = sm + L_H2 + ((t + 1) & 1) * TR_SPX * TD;
        float* h2 = sm + L_H2 + (t & 1) * TR_SPX * TD;
        // gathers: wave w fetches half gf = (w >> 2) of sentence (w & 3)'s vector
        const int gs = wave & 3, gf = wave >> 2;
        const bool gon = gs < ns;
        // ---- 0) prenet L1 of this step (+ the continue flags), from step t-1
        if (t > 0) {
            if (gon) {
                float v3[3];
                const bool ok = sweep<3>(Gp + G_PRE1, Ep + P_PRE1, v3, [&](int i) {
                    if (i < 2) return gs * T_PRE1 + gf * 128 + ln + 64 * i;
                    return (wave == 0 && ln < ns) ? TR_SPX * T_PRE1 + ln : -1;
                }, tmo, fsl);
                pre1[gs * T_PRE1 + gf * 128 + lane] = v3[0];
                pre1[gs * T_PRE1 + gf * 128 + 64 + lane] = v3[1];
                if (wave == 0 && lane < ns) dn[lane] = v3[2] == 0.f ? 1 : 0;
                if (!ok && lane == 0) { ctl[0] = 1; fail(a.status, 1); }
            }
            __syncthreads();
            if (ctl[0]) return;
            bool all = true;
            for (int s = 0; s < ns; ++s) all = all && dn[s];
            MARK(0);
            if (all) break;
        }
        // ---- 1) prenet L2 (waves 0-3, row 4r + w) -> xa[s][0:128]
        if (wave < 4) {
            float p[TR_SPX];
            dot4(p, w2q, pre1, T_PRE1, lane);
            const float v = to_lanes(p, lane);
            if (lane < ns) publish(G + G_PRE2 + lane * T_PRE2 + r2, E + P_PRE2, fmaxf(v + bias[14], 0.f));
        }
        if (gon) {
            float v1[1];
            const bool ok = sweep<1>(G + G_PRE2, E + P_PRE2, v1, [&](int i) { return gs * T_PRE2 + gf * 64 + ln; }, tmo, fsl);
            xa[gs * TXA + gf * 64 + lane] = v1[0];
            if (!ok && lane == 0) { ctl[0] = 1; fail(a.status, 2); }
        }
        __syncthreads();
        if (ctl[0]) return;
        MARK(1);
        // ---- 2) attention GRU, unit U: x = [prenet | ctx_{t-1}], h = h_att_{t-1} (:370); the four
        // sentences' dot products interleaved, sentence s finished by lane s
        {
            float v[4 * TR_SPX];  // [gate r, z, n_x, n_h][sentence]
#pragma unroll
            for (int s = 0; s < TR_SPX; ++s) {
                const float2 xp = ld2(xa + s * TXA + 2 * lane);
                const float4 xc = ld4(xa + s * TXA + T_PRE2 + 4 * lane);
                const float4 hv = ld4(hatt_prev + s * TD + 4 * lane);
                const float x6[6] = {xp.x, xp.y, xc.x, xc.y, xc.z, xc.w};
                const float h4[4] = {hv.x, hv.y, hv.z, hv.w};
                float pr = 0.f, pz = 0.f, pn = 0.f, qn = 0.f;
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    pr = fmaf(axr[i], x6[i], pr);
                    pz = fmaf(axz[i], x6[i], pz);
                    pn = fmaf(axn[i], x6[i], pn);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    pr = fmaf(ahr[i], h4[i], pr);
                    pz = fmaf(ahz[i], h4[i], pz);
                    qn = fmaf(ahn[i], h4[i], qn);
                }
                v[s] = pr;
                v[TR_SPX + s] = pz;
                v[2 * TR_SPX + s] = pn;
                v[3 * TR_SPX + s] = qn;
            }
            const float tot = xreduce<4 * TR_SPX>(v, lane);  // value k = 4 gate + s in lane 4k
            const float R = __shfl(tot, 4 * (lane & 3), 64), Z = __shfl(tot, 4 * (4 + (lane & 3)), 64),
                        N = __shfl(tot, 4 * (8 + (lane & 3)), 64), Q = __shfl(tot, 4 * (12 + (lane & 3)), 64);
            if (lane < ns) {
                const float rg = sigmoid_cell(R + bias[0]);
                const float zg = sigmoid_cell(Z + bias[1]);
                const float ng = tanh_cell((N + bias[2]) + rg * (Q + bias[3]));
                publish(G + G_HATT + lane * TD + U, E + P_HATT, (hatt_prev[lane * TD + U] - ng) * zg + ng);
            }
        }
        MARK(12);
        if (gon) {
            float v2[2];
            const bool ok = sweep<2>(G + G_HATT, E + P_HATT, v2, [&](int i) { return gs * TD + gf * 128 + ln + 64 * i; }, tmo, fsl);
            hatt[gs * TD + gf * 128 + lane] = v2[0];
            hatt[gs * TD + gf * 128 + 64 + lane] = v2[1];
            if (!ok && lane == 0) { ctl[0] = 1; fail(a.status, 3); }
        }
        __syncthreads();
        if (ctl[0]) return;
        MARK(2);
        // ---- 3) query_layer (waves 4-7, row 4r + w - 4) over h_att_t (common_layers.py:179)
        if (wave >= 4) {
            float p[TR_SPX];
            dot4(p, w2q, hatt, TD, lane);
            const float v = to_lanes(p, lane);
            if (lane < ns) publish(G + G_Q + lane * ADIM + r2, E + P_Q, v);
        }
        if (att_on && wave < 2) {
            float v1[1];
            const bool ok = sweep<1>(G + G_Q, E + P_Q, v1, [&](int i) { return sa * ADIM + wave * 64 + ln; }, tmo, fsl);
            q[wave * 64 + lane] = v1[0];
            if (!ok && lane == 0) { ctl[0] = 1; fail(a.status, 4); }
        }
        __syncthreads();
        if (ctl[0]) return;
        MARK(3);
        // ---- 4) attention over this CU's 32 positions (common_layers.py:178-182, 199-217, 241-243)
        if (att_on) {
            const int jl = tid >> 4, dc = tid & 15;
            float e = 0.f;
            const float* pv = Ps + jl * ADIM + dc * 8;
            const float* vv = sm + L_V + dc * 8;
            const float* qq = q + dc * 8;
#pragma unroll
            for (int dd = 0; dd < 8; ++dd) e += vv[dd] * tanh_fast(qq[dd] + pv[dd]);
            e = row_sum16(e);
            if (dc == 15) {
                const int j = j0 + jl;
                float w = 0.f;
                if (j < La) {
                    const float sg = sigmoidf_(e + vb);
                    const float prev = jl > 0 ? al[jl - 1] : al[TR_PPC];
                    const float mix = __fadd_rn(__fadd_rn(__fmul_rn(0.5f, al[jl]), __fmul_rn(0.5f, prev)), 1e-8f);
                    w = __fmul_rn(mix, sg);
                }
                wj[jl] = w;
            }
            __syncthreads();
            {
                const int d = tid & (TD - 1), half = tid >> 8;
                float acc = 0.f;
#pragma unroll
                for (int k = 0; k < 16; ++k) acc = fmaf(wj[16 * half + k], Es[(16 * half + k) * TD + d], acc);
                red[half * 280 + d] = acc;
            }
            __syncthreads();
            u64* gp = G + G_ATTP + (sa * TR_CPS + ka) * ATTP_W;
            if (tid < TD) {
                publish(gp + tid, E + P_ATTP, red[tid] + red[280 + tid]);
            } else if (tid == TD) {
                float sw = 0.f;
                for (int k = 0; k < TR_PPC; ++k) sw += wj[k];  // index order
                publish(gp + TD, E + P_ATTP, sw);
            } else if (tid == TD + 1) {
                publish(gp + TD + 1, E + P_ATTP, wj[TR_PPC - 1]);  // next slice's alpha_{j-1}
            } else if (tid == TD + 2) {
                const int jt = La - 1 - j0;
                publish(gp + TD + 2, E + P_ATTP, (jt >= 0 && jt < TR_PPC) ? wj[jt] : 0.f);
            }
            MARK(4);
            // the sentence's first CU adds the 8 slices' partials in slice order
            if (ka == 0) {
                float v8[TR_CPS];
                bool ok = true;
                if (tid < ATTP_W - 1)
                    ok = sweep<TR_CPS>(G + G_ATTP + sa * TR_CPS * ATTP_W, E + P_ATTP, v8,
                                       [&](int i) { return i * ATTP_W + tid; }, tmo, fsl);
                __syncthreads();  // red is rewritten below
                if (tid < ATTP_W - 1) {
                    float sum = 0.f;
#pragma unroll
                    for (int k = 0; k < TR_CPS; ++k) sum += v8[k];
                    red[tid] = sum;
                    if (tid == TD + 1)
#pragma unroll
                        for (int k = 0; k < TR_CPS; ++k) red[280 + k] = v8[k];
                }
                if (!ok) { ctl[0] = 1; fail(a.status, 5); }
                __syncthreads();
                if (ctl[0]) return;
                const float W = red[TD];
                u64* gc = G + G_CTXF + sa * CTXF_W;
                if (tid < TD) publish(gc + tid, E + P_CTXF, red[tid] / W);           // context
                else if (tid == TD) publish(gc + TD, E + P_CTXF, W);                  // normaliser
                else if (tid == TD + 1) publish(gc + TD + 1, E + P_CTXF, red[TD + 2] / W);  // alpha[L-1]
                else if (tid < TD + 2 + TR_CPS) {
                    const int k = tid - TD - 2;
                    publish(gc + TD + 2 + k, E + P_CTXF, red[280 + k] / W);         // alpha at slice ends
                }
                MARK(5);
            }
        }
        // everyone: the contexts, normalisers, tails and boundary alphas of the group's sentences
        if (gon) {
            float v3[3];
            const bool ok = sweep<3>(G + G_CTXF, E + P_CTXF, v3, [&](int i) {
                if (i < 2) return gs * CTXF_W + gf * 128 + ln + 64 * i;
                return (gf == 1 && ln < 2 + TR_CPS) ? gs * CTXF_W + TD + ln : -1;
            }, tmo, fsl);
            xa[gs * TXA + T_PRE2 + gf * 128 + lane] = v3[0];
            xa[gs * TXA + T_PRE2 + gf * 128 + 64 + lane] = v3[1];
            if (gf == 1) {
                if (lane == 0) nrm[gs] = v3[2];
                if (lane == 1) tl[gs] = v3[2];
                if (lane >= 2 && lane < 2 + TR_CPS) bnd[gs * TR_CPS + lane - 2] = v3[2];
            }
            if (!ok && lane == 0) { ctl[0] = 1; fail(a.status, 6); }
        }
        __syncthreads();
        if (ctl[0]) return;
        MARK(6);
        if (att_on) {
            // this step's alpha at this CU's positions (next step's prev_alpha) and the alignment row
            if (tid < TR_PPC) {
                const float w = wj[tid] / nrm[sa];
                al[tid] = w;
                const int j = j0 + tid;
                if (!dn[sa] && t < a.hist_cap && j < a.Lalign)
                    a.align_hist[((int64_t)ba * a.hist_cap + t) * a.Lalign + j] = j < La ? w : 0.f;
            }
            if (tid == TR_PPC) al[TR_PPC] = ka > 0 ? bnd[sa * TR_CPS + ka - 1] : 0.f;
        }
        // ---- 5) project_to_decoder_in, row U, over [h_att_t | ctx_t] (:373-375)
        {
            float p[TR_SPX];
#pragma unroll
            for (int s = 0; s < TR_SPX; ++s) {
                const float4 h = ld4(hatt + s * TD + 4 * lane);
                const float4 x = ld4(xa + s * TXA + T_PRE2 + 4 * lane);
                p[s] = fmaf(wp[7], x.w, fmaf(wp[6], x.z, fmaf(wp[5], x.y, fmaf(wp[4], x.x,
                       fmaf(wp[3], h.w, fmaf(wp[2], h.z, fmaf(wp[1], h.y, wp[0] * h.x)))))));
            }
            const float v = to_lanes(p, lane);
            if (lane < ns) publish(G + G_DIN + lane * TD + U, E + P_DIN, v + bias[12]);
        }
        if (gon) {
            float v2[2];
            const bool ok = sweep<2>(G + G_DIN, E + P_DIN, v2, [&](int i) { return gs * TD + gf * 128 + ln + 64 * i; }, tmo, fsl);
            din[gs * TD + gf * 128 + lane] = v2[0];
            din[gs * TD + gf * 128 + 64 + lane] = v2[1];
            if (!ok && lane == 0) { ctl[0] = 1; fail(a.status, 7); }
        }
        __syncthreads();
        if (ctl[0]) return;
        MARK(7);
        // ---- 6, 7) decoder GRUs with residuals (:377-382): x -> h' = GRU(x, h); out = h' + x
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const float* X = g == 0 ? din : d1;
            const float* Hp = g == 0 ? h1_prev : h2_prev;
            float* Hn = g == 0 ? h1 : h2;
            float* Dn = g == 0 ? d1 : d2;
            u64* gg = G + (g == 0 ? G_H1 : G_H2);
            const unsigned tg = E + (g == 0 ? P_H1 : P_H2);
            {
                float v[4 * TR_SPX];
#pragma unroll
                for (int s = 0; s < TR_SPX; ++s) {
                    const float4 xv = ld4(X + s * TD + 4 * lane);
                    const float4 hv = ld4(Hp + s * TD + 4 * lane);
                    const float x4[4] = {xv.x, xv.y, xv.z, xv.w}, h4[4] = {hv.x, hv.y, hv.z, hv.w};
                    float pr = 0.f, pz = 0.f, pn = 0.f, qn = 0.f;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        pr = fmaf(gx[g][0][i], x4[i], pr);
                        pz = fmaf(gx[g][1][i], x4[i], pz);
                        pn = fmaf(gx[g][2][i], x4[i], pn);
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        pr = fmaf(gh[g][0][i], h4[i], pr);
                        pz = fmaf(gh[g][1][i], h4[i], pz);
                        qn = fmaf(gh[g][2][i], h4[i], qn);
                    }
                    v[s] = pr;
                    v[TR_SPX + s] = pz;
                    v[2 * TR_SPX + s] = pn;
                    v[3 * TR_SPX + s] = qn;
                }
                const float tot = xreduce<4 * TR_SPX>(v, lane);
                const float R = __shfl(tot, 4 * (lane & 3), 64), Z = __shfl(tot, 4 * (4 + (lane & 3)), 64),
                            N = __shfl(tot, 4 * (8 + (lane & 3)), 64), Q = __shfl(tot, 4 * (12 + (lane & 3)), 64);
                if (lane < ns) {
                    const float rg = sigmoid_cell(R + bias[4 + 4 * g]);
                    const float zg = sigmoid_cell(Z + bias[5 + 4 * g]);
                    const float ng = tanh_cell((N + bias[6 + 4 * g]) + rg * (Q + bias[7 + 4 * g]));
                    const float hn = (Hp[lane * TD + U] - ng) * zg + ng;
                    publish(gg + lane * TD + U, tg, hn);
                    publish(gg + TR_SPX * TD + lane * TD + U, tg, hn + X[lane * TD + U]);
                }
            }
            MARK(13 + g);
            if (gon) {
                float v4[4];
                const bool ok = sweep<4>(gg, tg, v4, [&](int i) {
                    return (i < 2 ? 0 : TR_SPX * TD) + gs * TD + gf * 128 + ln + 64 * (i & 1);
                }, tmo, fsl);
                Hn[gs * TD + gf * 128 + lane] = v4[0];
                Hn[gs * TD + gf * 128 + 64 + lane] = v4[1];
                Dn[gs * TD + gf * 128 + lane] = v4[2];
                Dn[gs * TD + gf * 128 + 64 + lane] = v4[3];
                if (!ok && lane == 0) { ctl[0] = 1; fail(a.status, 10 + g); }
            }
            __syncthreads();
            if (ctl[0]) return;
            MARK(8 + g);
        }
        // ---- 8) output = sigmoid(proj_to_mel(decoder_output)), rows m0, m1 (:385-386) -> history
        {
            float p[2 * TR_SPX];  // [row m0, m1][sentence]
            const float4 w0 = ld4(wm + 4 * lane), w1_ = ld4(wm + 256 + 4 * lane);
#pragma unroll
            for (int s = 0; s < TR_SPX; ++s) {
                const float4 x = ld4(d2 + s * TD + 4 * lane);
                p[s] = fmaf(w0.w, x.w, fmaf(w0.z, x.z, fmaf(w0.y, x.y, w0.x * x.x)));
                p[TR_SPX + s] = fmaf(w1_.w, x.w, fmaf(w1_.z, x.z, fmaf(w1_.y, x.y, w1_.x * x.x)));
            }
            const float tot = xreduce<2 * TR_SPX>(p, lane);  // value k in lane 8k
            const float v0 = __shfl(tot, 8 * (lane & 3), 64), v1 = __shfl(tot, 8 * (4 + (lane & 3)), 64);
            if (lane < ns) {  // rows past nmel publish 0 (the gather reads all TR_NMEL_MAX)
                const int b = b0 + lane;
                const float o0 = m0 < nmel ? sigmoidf_(v0 + bm0) : 0.f;
                const float o1 = m1 < nmel ? sigmoidf_(v1 + bm1) : 0.f;
                publish(G + G_MEL + lane * TR_NMEL_MAX + m0, E + P_MEL, o0);
                publish(G + G_MEL + lane * TR_NMEL_MAX + m1, E + P_MEL, o1);
                if (t < a.hist_cap) {
                    if (m0 < nmel) a.mel_hist[((int64_t)b * a.hist_cap + t) * nmel + m0] = o0;
                    if (m1 < nmel) a.mel_hist[((int64_t)b * a.hist_cap + t) * nmel + m1] = o1;
                }
            }
        }
        MARK(15);
        if (gon) {
            float v4[4];
            const bool ok = sweep<4>(G + G_MEL, E + P_MEL, v4, [&](int i) {
                return gs * TR_NMEL_MAX + gf * 256 + ln + 64 * i;
            }, tmo, fsl);
#pragma unroll
            for (int i = 0; i < 4; ++i) mel[gs * TR_NMEL_MAX + gf * 256 + lane + 64 * i] = v4[i];
            if (!ok && lane == 0) { ctl[0] = 1; fail(a.status, 12); }
        }
        __syncthreads();
        if (ctl[0]) return;
        MARK(10);
        // ---- 9) stopnet over [decoder_output | output] + stop rule (:388-393, 459-469): rank 0, wave s
        // for sentence s, published before the prenet rows so it is off the critical path
        if (r == 0 && wave < ns) {
            const int s = wave;
            float p = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) p = fmaf(sm[L_STOP + lane + 64 * i], d2[s * TD + lane + 64 * i], p);
#pragma unroll
            for (int i = 0; i < 8; ++i) p = fmaf(sm[L_STOP + TD + lane + 64 * i], mel[s * TR_NMEL_MAX + lane + 64 * i], p);
            p = wave_sum_dpp(p);
            if (lane == 0) {
                const int b = b0 + s;
                int nd = dn[s];
                if (!nd) {
                    const float stv = sigmoidf_(p + bstop);
                    if (t < a.hist_cap) a.stop_hist[(int64_t)b * a.hist_cap + t] = stv;
                    // t = step + 1 after the append: t > L/4 and (stop > 0.6 [float32] or
                    // alignment[-1] > 0.6 [double]); elif t > max_decoder_steps
                    const int t1 = t + 1;
                    if ((4 * t1 > Ls[s] && (stv > 0.6f || (double)tl[s] > 0.6)) || t1 > a.max_steps) {
                        nd = 1;
                        a.done[b] = 1;
                        a.n_steps[b] = t1;
                    }
                }
                publish(G + G_PRE1 + TR_SPX * T_PRE1 + s, E + P_PRE1, nd ? 0.f : 1.f);
            }
        }
        // prenet L1 of step t+1, row U (memory = this output, memory_size == r: :396-404)
        {
            float p[TR_SPX];
            const float4 wa = ld4(w1 + 4 * lane), wb = ld4(w1 + 256 + 4 * lane);
#pragma unroll
            for (int s = 0; s < TR_SPX; ++s) {
                const float4 xa_ = ld4(mel + s * TR_NMEL_MAX + 8 * lane);
                const float4 xb_ = ld4(mel + s * TR_NMEL_MAX + 8 * lane + 4);
                p[s] = fmaf(wb.w, xb_.w, fmaf(wb.z, xb_.z, fmaf(wb.y, xb_.y, fmaf(wb.x, xb_.x,
                       fmaf(wa.w, xa_.w, fmaf(wa.z, xa_.z, fmaf(wa.y, xa_.y, wa.x * xa_.x)))))));
            }
            const float v = to_lanes(p, lane);
            if (lane < ns) publish(G + G_PRE1 + lane * T_PRE1 + U, E + P_PRE1, fmaxf(v + bias[13], 0.f));
        }
        MARK(11);
    }
    __syncthreads();
    if (prof && tid < TR_PHASES) a.prof[r * TR_PHASES + tid] = (long long)pacc[tid];
#undef MARK
}

}  // namespace

size_t tres_granules() { return (size_t)G_TOTAL + 2; }
size_t tres_smem_bytes() { return (size_t)L_TOTAL * sizeof(float); }

hipError_t tres_prepare() {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&tacotron_resident_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)tres_smem_bytes());
}

hipError_t launch_tacotron_resident(const TResArgs& a, hipStream_t s, bool* launched) {
    *launched = false;
    if (a.B < 1 || a.B > TR_SPX * TR_GROUPS || a.nmel > TR_NMEL_MAX || a.Lalign > TR_LMAX || a.max_steps > 1000)
        return hipErrorInvalidValue;
    TResArgs arg = a;
    void* args[] = {&arg};
    return launch_persistent(reinterpret_cast<const void*>(&tacotron_resident_kernel), dim3(TR_CUS), dim3(TR_THREADS),
                             args, tres_smem_bytes(), s, launched);
}

}  // namespace tts

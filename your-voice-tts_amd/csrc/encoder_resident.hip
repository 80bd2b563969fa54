// Resident batch-1 encoder BiLSTM (Encoder.inference's nn.LSTM, layers/tacotron2.py:56-61, 82):
// the whole recurrence of both directions as ONE launch instead of L dependent step launches.
//
// 256 workgroups are launched; each reads its XCC id and the 256-entry table of all of them.  The
// forward direction takes the first 32 workgroups (by index) of workgroup 0's XCD, the backward
// direction the first 32 of the next XCD (slot = rank in the XCD); the rest exit.  A role holds
// W_hh rows of 8 hidden units (x 4 gates, 32 rows x 256, 32 KiB) in VGPRs; thread (row r = tid / 8,
// k slice q = tid % 8) owns W_hh[row][32q .. 32q+32).  Rows are unit-major (r = 4 u + gate) so
// the 32 lanes of a unit hold its 4 gate sums after the 8-lane reduction, and one lane per unit
// updates (c, h) like the sgemm ENC_LSTM epilogue.  Per step every role publishes its 8 h values
// as 8-byte {tag, value} granules with a workgroup-scope store (the line stays in the XCD's L2)
// and gathers its direction's 256 values with agent-scope loads: XCD-local hand-offs, no fences.
// Waits are bounded (status on timeout).
//
// Geometry (ENC_RES_WIDE, measured at L = 100 per encoder call, round 5): 0 = both directions on
// one XCD, 16 workgroups x 512 threads (32 units each): 257 us; 1 = one XCD, 32 x 256: 221 us;
// 2 = one XCD per direction, 64 x 128 (4 k slices per row): 202-212 us; 3 (default) = the same
// with 8 k slices per row, 64 x 256 (every SIMD of the CU issues): 191-203 us.  The step is the
// dot products' issue plus the XCD-local edge, so spreading the rows over more SIMDs pays until
// the edge dominates.
#include "encoder_resident.h"

#ifndef ENC_SLEEP
#define ENC_SLEEP 1  // s_sleep between hand-off polls
#endif

namespace tts {
namespace {

typedef unsigned long long u64;
typedef __attribute__((address_space(1))) u64 gu64;
typedef __attribute__((address_space(1))) int gint;

#ifndef ENC_RES_WIDE
#define ENC_RES_WIDE 3
#endif
constexpr int ER_THREADS = ENC_RES_WIDE == 2 ? 128 : ENC_RES_WIDE == 1 || ENC_RES_WIDE == 3 ? 256 : 512;
constexpr int ER_SLOTS = ENC_RES_WIDE >= 2 ? 32 : ENC_RES_WIDE ? 16 : 8;  // workgroups per direction
constexpr int ER_KS = ENC_RES_WIDE == 3 ? 8 : 4;                           // threads (k slices) per gate row
constexpr int ER_UNITS = ER_THREADS / (4 * ER_KS);                         // hidden units per workgroup
constexpr bool ER_SPLIT = ENC_RES_WIDE >= 2;  // one XCD per direction (else both on CU 0's XCD)
constexpr int H = 256, G4 = 4 * H;
constexpr int ER_NW = H / 4 / ER_KS;  // float4 weights per thread
constexpr int GR_TABLE = 0, GR_H = 256;  // granules: table [256], h [2 parity][2 dir][256]

__device__ __forceinline__ void pub_dev(u64* g, unsigned tag, float v) {
    __hip_atomic_store((gu64*)g, ((u64)tag << 32) | (u64)__float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void pub_xcd(u64* g, unsigned tag, float v) {
    __hip_atomic_store((gu64*)g, ((u64)tag << 32) | (u64)__float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ u64 peek(u64* g) {
    return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one wave: lane l polls granules base + 4l .. 4l+3 until every tag matches
__device__ __forceinline__ bool sweep4(u64* g, unsigned tag, float (&v)[4], long long tmo) {
    const int lane = threadIdx.x & 63;
    long long t_end = 0;
    for (int spin = 0;; ++spin) {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const u64 x = peek(g + lane * 4 + i);
            v[i] = __uint_as_float((unsigned)x);
            ok = ok && (unsigned)(x >> 32) == tag;
        }
        if (__all(ok)) return true;
        if (spin == 0) t_end = (long long)wall_clock64() + tmo;
        else if ((spin & 31) == 0 && (long long)wall_clock64() > t_end) return false;
        if (ENC_SLEEP) __builtin_amdgcn_s_sleep(ENC_SLEEP);
    }
}
// one lane polls the 16-byte granule pair `pair` (granules 2 pair, 2 pair + 1 of rsrc r) until
// both tags match (sc1 | volatile buffer loads: L1 bypass, re-issued every poll)
typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bool sweep_pair(__amdgpu_buffer_rsrc_t r, int pair, unsigned tag, float (&v)[2], long long tmo) {
    long long t_end = 0;
    for (int spin = 0;; ++spin) {
        const u32x4_ x = __builtin_bit_cast(u32x4_, __builtin_amdgcn_raw_buffer_load_b128(r, pair * 16, 0, (int)0x80000010u));
        v[0] = __uint_as_float(x.x);
        v[1] = __uint_as_float(x.z);
        if (__all(x.y == tag && x.w == tag)) return true;
        if (spin == 0) t_end = (long long)wall_clock64() + tmo;
        else if ((spin & 31) == 0 && (long long)wall_clock64() > t_end) return false;
        if (ENC_SLEEP) __builtin_amdgcn_s_sleep(ENC_SLEEP);
    }
}
__device__ __forceinline__ float dot4(float4 w, float4 x, float acc) {
    acc = fmaf(w.x, x.x, acc);
    acc = fmaf(w.y, x.y, acc);
    acc = fmaf(w.z, x.z, acc);
    return fmaf(w.w, x.w, acc);
}

__global__ __launch_bounds__(ER_THREADS, 1) void encoder_resident_kernel(const EncResArgs a) {
    const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    __shared__ __align__(16) float hsb[2][H];  // h_{s-1} by step parity (the gather fills the other)
    __shared__ int info[4];
    // ---- roles from the XCD table
    int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7;
    const unsigned setup_tag = (a.salt << 14) | 0x3FFFu;
    if (tid == 0) pub_dev(a.gran + GR_TABLE + c, setup_tag, __int_as_float(xcc));
    if (wave == 0) {
        float v[4];
        const bool ok = sweep4(a.gran + GR_TABLE, setup_tag, v, a.tmo);
        const int xref = __builtin_amdgcn_readfirstlane(__float_as_int(v[0]) & 7);
        // ER_SPLIT: the backward direction on the XCD of the first workgroup off xref's XCD
        int first = 1 << 20;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const u64 m = __ballot((__float_as_int(v[i]) & 7) != xref);
            if (m) first = min(first, 4 * __builtin_ctzll(m) + i);
        }
        const int xref1 = ER_SPLIT && first < 256 ? __float_as_int(__uint_as_float((unsigned)peek(a.gran + GR_TABLE + first))) & 7 : xref;
        const int xmine = ER_SPLIT && xcc == xref1 ? xref1 : xref;
        int rank = 0, nref = 0, nref1 = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int x = __float_as_int(v[i]) & 7;
            nref += __popcll(__ballot(x == xref));
            nref1 += __popcll(__ballot(x == xref1));
            rank += __popcll(__ballot(x == xmine && lane * 4 + i < c));
        }
        if (ER_SPLIT) {
            if (xref1 == xref) nref = 0;  // one XCD only: no placement for the split form
            nref = min(nref, nref1) * 2;  // the roles need ER_SLOTS on each of the two XCDs
        }
        if (lane == 0) {
            info[0] = ok ? 1 : 0;
            info[1] = !ER_SPLIT ? (xcc == xref ? rank : -1)
                                : xcc == xref ? rank : xcc == xref1 ? ER_SLOTS + rank : -1;
            if (ER_SPLIT && rank >= ER_SLOTS) info[1] = -1;
            info[2] = nref;
            info[3] = 0;
            // status word = salt << 8 | code (res_status_code): no clearing between launches
            if (!ok) __hip_atomic_store((gint*)a.status, (int)((a.salt << 8) | 6u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (nref < 2 * ER_SLOTS && c == 0)
                __hip_atomic_store((gint*)a.status, (int)((a.salt << 8) | (unsigned)ENC_RES_STATUS_PLACEMENT), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    const int role = info[1];
    if (!info[0] || info[2] < 2 * ER_SLOTS || role < 0 || role >= 2 * ER_SLOTS) return;
    const int dir = role / ER_SLOTS, slot = role % ER_SLOTS;
    const int row = tid / ER_KS, kq = tid % ER_KS;  // row = 4 * unit_local + gate
    const int ul = row >> 2, gate = row & 3;
    const int unit = slot * ER_UNITS + ul;
    float4 w[ER_NW];
    const float4* wp = a.w + ((size_t)(dir * ER_SLOTS + slot) * ER_NW) * ER_THREADS + tid;
#pragma unroll
    for (int i = 0; i < ER_NW; ++i) w[i] = wp[(size_t)i * ER_THREADS];
    // initial state
    for (int k = tid; k < H; k += ER_THREADS) hsb[0][k] = a.h0 ? a.h0[dir * a.hdir + k] : 0.f;
    float cs = 0.f;  // cell of `unit` (lanes with row & 3 == 0 && kq == 0)
    if (a.c0) cs = a.c0[dir * a.hdir + unit];
    float hlast = 0.f;
    const int L = a.L;
    auto xi_at = [&](int s) -> float {
        const int pos = dir == 0 ? s : L - 1 - s;
        return a.xi[(int64_t)pos * (2 * G4) + dir * G4 + gate * H + unit];
    };
    float xcur = L > 0 ? xi_at(0) : 0.f;
    // the h granules [2 parity][2 dir][256] as 16-byte pairs (buffer loads, sc1)
    const auto gr = __builtin_amdgcn_make_buffer_rsrc(a.gran + GR_H, (short)0, 2 * 2 * H * 8, 0x00020000);
    __syncthreads();
    for (int s = 0; s < L; ++s) {
        const float xnext = s + 1 < L ? xi_at(s + 1) : 0.f;  // in flight during this step
        const float* hs = hsb[s & 1];
        // four independent accumulators (a 16-FMA dependency chain each instead of one of 64)
        float a4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < ER_NW; ++i)
            a4[i & 3] = dot4(w[i], *reinterpret_cast<const float4*>(hs + kq * (H / ER_KS) + 4 * i), a4[i & 3]);
        float acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
        // sum over the row's k slices, then gate pre-activation
        acc += dpp_move<0xB1, 0xf>(acc, 0.f);  // quad_perm [1,0,3,2]
        acc += dpp_move<0x4E, 0xf>(acc, 0.f);  // quad_perm [2,3,0,1]
        if constexpr (ER_KS == 8) acc += dpp_move<0x141, 0xf>(acc, 0.f);  // row_half_mirror: the other quad
        const float pre = acc + xcur;
        const float act = gate == 2 ? tanh_cell(pre) : sigmoid_cell(pre);
        float f, g, o;
        if constexpr (ER_KS == 4) {
            f = dpp_move<0x104, 0xf>(act, 0.f);  // row_shl:4  -> gate 1 of this unit
            g = dpp_move<0x108, 0xf>(act, 0.f);  // row_shl:8  -> gate 2
            o = dpp_move<0x10C, 0xf>(act, 0.f);  // row_shl:12 -> gate 3
        } else {  // gate rows 8 lanes apart: gates 2, 3 sit in the next DPP row (lane ^ 16 swizzle)
            f = dpp_move<0x108, 0xf>(act, 0.f);  // row_shl:8 -> gate 1
            g = __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, act), 0x401F));
            o = __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, f), 0x401F));
        }
        const int par = s & 1;
        u64* gh = a.gran + GR_H + (par * 2 + dir) * H;
        if ((tid & (4 * ER_KS - 1)) == 0) {
            cs = f * cs + act * g;  // c' = s(f) c + s(i) tanh(g)
            const float h = o * tanh_cell(cs);
            hlast = h;
            pub_xcd(gh + unit, (a.salt << 14) | (unsigned)(s + 1), h);
            const int pos = dir == 0 ? s : L - 1 - s;
            a.out[(int64_t)pos * (2 * H) + dir * H + unit] = h;
        }
        xcur = xnext;
        if (wave < 2) {
            // the direction's 256 h values: one 16-byte granule pair per lane on waves 0 and 1
            // (one load instruction per poll instead of four on one wave)
            float v[2];
            const int pr = wave * 64 + lane;
            for (int i = 0; i < a.first_sleep; ++i) __builtin_amdgcn_s_sleep(1);
            const bool ok = sweep_pair(gr, ((par * 2 + dir) * H) / 2 + pr, (a.salt << 14) | (unsigned)(s + 1), v, a.tmo);
            if (!ok) {
                if (lane == 0)
                    __hip_atomic_store((gint*)a.status, (int)((a.salt << 8) | 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                info[3] = 1;
            }
            *reinterpret_cast<float2*>(hsb[(s + 1) & 1] + pr * 2) = float2{v[0], v[1]};
        }
        __syncthreads();
        if (info[3] == 1) return;
    }
    if ((tid & (4 * ER_KS - 1)) == 0 && L > 0) {
        a.h_fin[dir * a.hdir + unit] = hlast;
        a.c_fin[dir * a.hdir + unit] = cs;
    }
}

// ---------------------------------------------------------------- batched form (B >= 2)
// XCD x: direction x & 1, sentences [g G, g G + G) with g = x >> 1 and G = ceil(B / 4).  Workgroup
// of rank r (in its XCD) owns hidden units [8 r, 8 r + 8): W_hh rows j = 4 u + gate (u < 8) as two
// 16-row MFMA A tiles.  Per step s, wave w multiplies tile w & 1 over k-steps [16 (w >> 1), +16)
// (v_mfma_f32_16x16x4_f32, A = W rows in registers, B = h_{s-1}^T of the group's 16 sentence
// columns from LDS); the 4 partial tiles of each row tile are summed in wave order through LDS;
// waves 0 / 1 then hold, per lane, the 4 gate sums of one (unit, sentence) and update (c, h)
// exactly as the ENC_LSTM epilogue (the input projection xi, both biases folded, added first);
// h goes to the output row and to an XCD-local {tag, h} granule; every wave then gathers the
// group's 256 x 16 granules into the other LDS h buffer.
constexpr int EB_THREADS = 512, EB_UNITS = 8, EB_G = 16, EB_LDH = H + 4;
constexpr int EB_GR_TABLE = 0, EB_GR_H = 256, EB_GR_PER = EB_G * H;  // per (parity, XCD)

__global__ __launch_bounds__(EB_THREADS, 1) void encoder_resident_batch_kernel(const EncResBatchArgs a) {
    const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    __shared__ __align__(16) float hs[2][EB_G][EB_LDH];  // h_{s-1} of the group's sentences, by parity
    __shared__ __align__(16) float red[8][64][4];        // partial gate tiles
    __shared__ int info[4];
    int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7;
    const unsigned setup_tag = (a.salt << 14) | 0x3FFFu;
    if (tid == 0) pub_dev(a.gran + EB_GR_TABLE + c, setup_tag, __int_as_float(xcc));
    if (wave == 0) {
        float v[4];
        const bool ok = sweep4(a.gran + EB_GR_TABLE, setup_tag, v, a.tmo);
        int rank = 0, nmin = 256;
        for (int x = 0; x < 8; ++x) {
            int cnt = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int xi = __float_as_int(v[i]) & 7;
                cnt += __popcll(__ballot(xi == x));
                if (x == xcc) rank += __popcll(__ballot(xi == x && lane * 4 + i < c));
            }
            nmin = min(nmin, cnt);
        }
        if (lane == 0) {
            info[0] = ok ? 1 : 0;
            info[1] = rank;
            info[2] = nmin;
            info[3] = 0;
            if (!ok) __hip_atomic_store((gint*)a.status, (int)((a.salt << 8) | 6u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (nmin < 32 && c == 0)
                __hip_atomic_store((gint*)a.status, (int)((a.salt << 8) | (unsigned)ENC_RES_STATUS_PLACEMENT), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    const int rank = info[1];
    if (!info[0] || info[2] < 32 || rank >= 32) return;
    const int dir = xcc & 1, G = (a.B + 3) / 4, b0 = (xcc >> 1) * G;
    const int nb = max(0, min(G, a.B - b0));  // sentences of this group
    if (nb == 0) return;
    int Lg = 0;
    for (int n = 0; n < nb; ++n) Lg = max(Lg, a.lens[b0 + n]);
    // A operands: tile rt = wave & 1, k-steps [16 kq, 16 kq + 16), kq = wave >> 1
    const int rt = wave & 1, kq = wave >> 1, row = lane & 15, q = lane >> 4;
    float wa[16];
    {
        const int j = rt * 16 + row, unit = rank * EB_UNITS + (j >> 2), gate = j & 3;
        const float* wr = a.whh + ((int64_t)dir * G4 + gate * H + unit) * H + q;
#pragma unroll
        for (int i = 0; i < 16; ++i) wa[i] = wr[4 * (16 * kq + i)];
    }
    for (int i = tid; i < 2 * EB_G * EB_LDH; i += EB_THREADS) (&hs[0][0][0])[i] = 0.f;
    // waves 0 / 1: lane's (unit, sentence n) and its cell
    const int n = lane & 15, unit = rank * EB_UNITS + 4 * rt + (lane >> 4);
    const int bsen = b0 + n, Ln = n < nb ? a.lens[bsen] : 0;
    float cs = 0.f, hprev = 0.f;
    float xg[4] = {0.f, 0.f, 0.f, 0.f};
    auto load_xi = [&](int s) {
        if (wave < 2 && s < Ln) {
            const int pos = dir ? Ln - 1 - s : s;
            const float* x = a.xi + ((int64_t)bsen * a.Tmax + pos) * (2 * G4) + dir * G4 + unit;
#pragma unroll
            for (int g = 0; g < 4; ++g) xg[g] = x[g * H];
        }
    };
    load_xi(0);
    __syncthreads();
    u64* gx = a.gran + EB_GR_H;  // + (parity * 8 + xcc) * EB_GR_PER
    for (int s = 0; s < Lg; ++s) {
        const int par = s & 1;
        // ---- partial gates: 16 MFMAs over this wave's k quarter, B = h^T[k][n] from LDS
        floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
        const float* hrow = &hs[par][n][0];
#pragma unroll
        for (int i = 0; i < 16; ++i) acc = mfma16x16x4(wa[i], hrow[4 * (16 * kq + i) + q], acc);
        *reinterpret_cast<floatx4*>(&red[wave][lane][0]) = acc;
        __syncthreads();
        if (wave < 2) {
            floatx4 sum = *reinterpret_cast<const floatx4*>(&red[rt][lane][0]);
#pragma unroll
            for (int w = 1; w < 4; ++w) sum += *reinterpret_cast<const floatx4*>(&red[rt + 2 * w][lane][0]);
            // D lane l holds rows 4 (l >> 4) + r of tile rt = gate r of unit 4 rt + (l >> 4), column n
            const bool act = s < Ln;
            const float gi = sum[0] + xg[0], gf = sum[1] + xg[1], gg = sum[2] + xg[2], go = sum[3] + xg[3];
            load_xi(s + 1);  // next step's input projection, in flight during the hand-off
            if (act) {
                const float c2 = sigmoid_cell(gf) * cs + sigmoid_cell(gi) * tanh_cell(gg);
                const float h = sigmoid_cell(go) * tanh_cell(c2);
                cs = c2;
                hprev = h;
                const int pos = dir ? Ln - 1 - s : s;
                a.out[((int64_t)bsen * a.Tmax + pos) * (2 * H) + dir * H + unit] = h;
            }
            // every lane publishes (idle sentences: their last h) so the gather sees every tag
            pub_xcd(gx + (int64_t)(par * 8 + xcc) * EB_GR_PER + n * H + unit, (a.salt << 14) | (unsigned)(s + 1), hprev);
        }
        // ---- gather the group's h_s into the other buffer: thread t sweeps granules t + 512 i
        {
            const unsigned tag = (a.salt << 14) | (unsigned)(s + 1);
            u64* gp = gx + (int64_t)(par * 8 + xcc) * EB_GR_PER;
            long long t_end = 0;
            constexpr int PER = EB_GR_PER / EB_THREADS;  // 8
            float v[PER];
            bool ok = true;
            for (int spin = 0;; ++spin) {
                ok = true;
#pragma unroll
                for (int i = 0; i < PER; ++i) {
                    const int gidx = tid + i * EB_THREADS, nn = gidx / H;
                    if (nn < nb) {
                        const u64 x = peek(gp + gidx);
                        v[i] = __uint_as_float((unsigned)x);
                        ok = ok && (unsigned)(x >> 32) == tag;
                    } else {
                        v[i] = 0.f;
                    }
                }
                if (__all(ok)) break;
                if (spin == 0) t_end = (long long)wall_clock64() + a.tmo;
                else if ((spin & 31) == 0 && (long long)wall_clock64() > t_end) break;
                if (ENC_SLEEP) __builtin_amdgcn_s_sleep(ENC_SLEEP);
            }
            if (!__all(ok)) {
                if (lane == 0) {
                    __hip_atomic_store((gint*)a.status, (int)((a.salt << 8) | 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    info[3] = 1;
                }
            }
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int gidx = tid + i * EB_THREADS;
                hs[par ^ 1][gidx / H][gidx % H] = v[i];
            }
        }
        __syncthreads();
        if (info[3]) return;
    }
}

__global__ void enc_res_pack_kernel(const float* whh_f, const float* whh_b, float4* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)2 * ER_SLOTS * ER_NW * ER_THREADS) return;
    const int tid = i % ER_THREADS, i4 = (i / ER_THREADS) % ER_NW, slot = (i / (ER_NW * ER_THREADS)) % ER_SLOTS;
    const int dir = i / (ER_NW * ER_THREADS * ER_SLOTS);
    const int row = tid / ER_KS, kq = tid % ER_KS, ul = row >> 2, gate = row & 3;
    const int ref = gate * H + slot * ER_UNITS + ul;
    const float* W = dir ? whh_b : whh_f;
    const float* p = W + (int64_t)ref * H + kq * (H / ER_KS) + 4 * i4;
    out[i] = float4{p[0], p[1], p[2], p[3]};
}

}  // namespace

size_t encoder_resident_batch_granules() { return EB_GR_H + (size_t)2 * 8 * EB_GR_PER + 2; }

hipError_t launch_encoder_resident_batch(const EncResBatchArgs& a, hipStream_t s, bool* launched) {
    *launched = false;
    if (a.B < 2 || a.B > 4 * EB_G) return hipErrorInvalidValue;
    EncResBatchArgs arg = a;
    void* args[] = {&arg};
    return launch_persistent(reinterpret_cast<const void*>(&encoder_resident_batch_kernel), dim3(256), dim3(EB_THREADS),
                             args, 0, s, launched);
}

size_t encoder_resident_weight_float4() { return (size_t)2 * ER_SLOTS * ER_NW * ER_THREADS; }
size_t encoder_resident_granules() { return GR_H + 4 * H + 2; }

hipError_t encoder_resident_pack(const float* whh_f, const float* whh_b, float4* out, hipStream_t s) {
    const int64_t n = (int64_t)encoder_resident_weight_float4();
    hipLaunchKernelGGL(enc_res_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, whh_f, whh_b, out);
    return hipGetLastError();
}

hipError_t launch_encoder_resident(const EncResArgs& a, hipStream_t s, bool* launched) {
    EncResArgs arg = a;
    void* args[] = {&arg};
    return launch_persistent(reinterpret_cast<const void*>(&encoder_resident_kernel), dim3(256), dim3(ER_THREADS),
                             args, 0, s, launched);
}

}  // namespace tts

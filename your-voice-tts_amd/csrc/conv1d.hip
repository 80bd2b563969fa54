// fp32 MFMA implicit-GEMM Conv1d (see conv1d.h).
//
//   out[b][t][co] = act( scale[co] * sum_{k<KW} sum_ci in[b][t+k-PAD][ci] * W[co][ci][k] + shift[co] ) (+ resid)
//
// GEMM view: M = frames, N = output channels, K = (tap, input channel).  A workgroup owns a
// BM x 64 output tile; per BK-channel K step it stages the BM+KW-1 input rows and the
// BK x KW x 64 weight slab in LDS (BK = 16 / 8 / 4 for KW <= 5 / 8 / 16: the slab stays <= 32 KB),
// then each wave issues v_mfma_f32_16x16x4_f32 on its (BM/WM) x (64/WN) sub-tile.  For KW <= 5
// one accumulator set per tap keeps the fp32 fma chains short (Cin long instead of KW*Cin); the
// long CBHG bank slabs (KW 8 / 16) accumulate every tap into one set (register budget).  Two tile
// shapes: BM=64 (2x2 waves of 32x32) for large batches (BM=32, 2x2 waves of 16x32, for the KW=5
// convs), BM=16 (1x4 waves of 16x16) so that a single sentence still spreads over >= 100 workgroups.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "conv1d.h"

namespace tts {

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int KW, int BM, int WM, int WN, bool SPLIT = false>
__global__ __launch_bounds__(256) void conv_kernel(const ConvArgs a, int nsplit = 1, int nb = 1) {
    constexpr int PAD = (KW - 1) / 2;
    constexpr int BK = KW <= 5 ? 16 : (KW <= 8 ? 8 : 4);
    constexpr int NACC = KW <= 5 ? KW : 1;  // accumulator sets (per tap for short kernels)
    constexpr int BN = CONV_BN;
    constexpr int TM = BM / WM / 16;
    constexpr int TN = BN / WN / 16;
    // 1-D grid, output-channel tile fastest: under round-robin workgroup placement XCD = bx % 8,
    // so every XCD works on a fixed set of channel tiles and its L2 keeps their weight slabs
    // (655 KB each at Cin = 512) across all the frame tiles it is given (speed only).
    const int ntl = a.co_pad / BN;
    const int Tt = a.Ttile ? a.Ttile : a.Tmax;
    const int mtiles = (Tt + BM - 1) / BM;
    // split-K: z-th slice of the K steps; the split index is the slowest grid coordinate
    const int ntiles_all = SPLIT ? (int)(gridDim.x / nsplit) : (int)gridDim.x;
    const int z = SPLIT ? (int)blockIdx.x / ntiles_all : 0;
    const int bx = SPLIT ? (int)blockIdx.x % ntiles_all : (int)blockIdx.x;
    const int ntile = bx % ntl;
    const int rest = bx / ntl;
    const int b = rest / mtiles;
    const int t0 = (rest % mtiles) * BM;
    const int c0 = ntile * BN;
    const int Tb = a.tmul > 1 ? a.T[b] * a.tmul : a.T[b];
    if (t0 >= Tb) return;
    const int64_t Tin = a.in_tmax ? a.in_tmax : a.Tmax;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wt = (wave / WN) * (BM / WM);
    const int wc = (wave % WN) * (BN / WN);
    // double-buffered LDS stages; the next K step's global loads are in registers while the
    // current step's MFMAs run (one barrier per K step)
    constexpr int XROWS = BM + KW - 1;
    constexpr int XN = XROWS * (BK / 4);     // float4 of input per stage
    constexpr int WN4 = BK * KW * (BN / 4);  // float4 of weights per stage
    constexpr int XR = (XN + 255) / 256, WR = (WN4 + 255) / 256;
    __shared__ float xs[2][XROWS][BK + 1];
    __shared__ __align__(16) float ws[2][BK][KW][BN];
    floatx4 acc[NACC][TM][TN];
#pragma unroll
    for (int k = 0; k < NACC; ++k)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[k][i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int* idsb = a.ids ? a.ids + (int64_t)b * a.Tmax : nullptr;
    float4 xr[XR], wr[WR];
    // global -> registers for the K step starting at input channel CI0, and registers -> LDS
    // stage BUF.  Every register of xr/wr is loaded unconditionally (clamped indices, a valid
    // dummy row for padding frames) so the arrays stay in VGPRs across the pipelined loop; a
    // guarded load leaves them partially defined and the compiler spills them to scratch.
#define CONV_GLOAD(CI0)                                                                                          \
    {                                                                                                            \
        const int ci0_ = (CI0);                                                                                  \
        _Pragma("unroll") for (int q = 0; q < XR; ++q) {                                                          \
            const int i = min(tid + q * 256, XN - 1);                                                            \
            const int r = i / (BK / 4), c4 = i % (BK / 4);                                                       \
            const int t = t0 - PAD + r;                                                                          \
            const bool ok = t >= 0 && t < Tb;                                                                    \
            const int tc = ok ? t : 0;                                                                           \
            const float* src = idsb ? a.table + (int64_t)idsb[tc] * a.Cin : a.in + ((int64_t)b * Tin + tc) * a.Cin; \
            float4 v = *reinterpret_cast<const float4*>(src + ci0_ + c4 * 4);                                    \
            if (a.pool2) { /* max(in[t], in[t+1]), in[T_b] = 0 */                                                \
                const bool ok1 = ok && t + 1 < Tb;                                                               \
                const float4 v1 = *reinterpret_cast<const float4*>(                                              \
                    a.in + ((int64_t)b * Tin + (ok1 ? t + 1 : tc)) * a.Cin + ci0_ + c4 * 4);                      \
                const float4 p1 = ok1 ? v1 : float4{0.f, 0.f, 0.f, 0.f};                                         \
                v = float4{fmaxf(v.x, p1.x), fmaxf(v.y, p1.y), fmaxf(v.z, p1.z), fmaxf(v.w, p1.w)};              \
            }                                                                                                    \
            xr[q] = ok ? v : float4{0.f, 0.f, 0.f, 0.f};                                                         \
        }                                                                                                        \
        _Pragma("unroll") for (int q = 0; q < WR; ++q) {                                                          \
            const int i = min(tid + q * 256, WN4 - 1);                                                           \
            const int c4 = i % (BN / 4), rk = i / (BN / 4); /* rk = ci_local * KW + k */                         \
            wr[q] = *reinterpret_cast<const float4*>(a.W + ((int64_t)(ci0_ * KW + rk)) * a.co_pad + c0 + c4 * 4); \
        }                                                                                                        \
    }
#define CONV_LSTORE(BUF)                                                                                         \
    {                                                                                                            \
        const int buf_ = (BUF);                                                                                  \
        _Pragma("unroll") for (int q = 0; q < XR; ++q) {                                                          \
            const int i = tid + q * 256;                                                                         \
            if (i < XN) {                                                                                        \
                const int r = i / (BK / 4), c4 = i % (BK / 4);                                                   \
                xs[buf_][r][c4 * 4 + 0] = xr[q].x;                                                               \
                xs[buf_][r][c4 * 4 + 1] = xr[q].y;                                                               \
                xs[buf_][r][c4 * 4 + 2] = xr[q].z;                                                               \
                xs[buf_][r][c4 * 4 + 3] = xr[q].w;                                                               \
            }                                                                                                    \
        }                                                                                                        \
        _Pragma("unroll") for (int q = 0; q < WR; ++q) {                                                          \
            const int i = tid + q * 256;                                                                         \
            if (i < WN4) {                                                                                       \
                const int c4 = i % (BN / 4), rk = i / (BN / 4);                                                  \
                *reinterpret_cast<float4*>(&ws[buf_][rk / KW][rk % KW][c4 * 4]) = wr[q];                         \
            }                                                                                                    \
        }                                                                                                        \
    }
    const int nsteps_all = a.Cin / BK;
    const int sbeg = SPLIT ? z * nsteps_all / nsplit : 0;
    const int send = SPLIT ? (z + 1) * nsteps_all / nsplit : nsteps_all;
    CONV_GLOAD(sbeg * BK);
    CONV_LSTORE(0);
    __syncthreads();
    const int row = lane & 15, kq = lane >> 4;
    for (int st = sbeg; st < send; ++st) {
        const int cur = (st - sbeg) & 1;
        CONV_GLOAD(min(st + 1, send - 1) * BK);  // the last step reloads itself (unused)
#pragma unroll
        for (int k = 0; k < KW; ++k) {
#pragma unroll
            for (int kk = 0; kk < BK; kk += 4) {
                float av[TM], bv[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) av[i] = xs[cur][wt + i * 16 + row + k][kk + kq];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv[j] = ws[cur][kk + kq][k][wc + j * 16 + row];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        floatx4& c = acc[NACC == 1 ? 0 : k][i][j];
                        c = mfma16x16x4(av[i], bv[j], c);
                    }
            }
        }
        CONV_LSTORE(cur ^ 1);  // the other stage: every wave left it at the previous barrier
        __syncthreads();
    }
#undef CONV_GLOAD
#undef CONV_LSTORE
    // epilogue: D lane l holds C[(l>>4)*4 + r][l&15]  (row = frame, col = channel)
    if (SPLIT && a.tickets) {
        // Fused reduction: the LAST of the tile's nsplit workgroups to arrive sums the partials in
        // split order and applies the epilogue (conv_reduce_kernel's arithmetic, bitwise).  Hand-off
        // (MI355X_MICROARCH.md, inter-workgroup visibility, sc1 table row 1): every partial is
        // stored write-through (16-byte sc1 stores: a lane's 4 rows are consecutive frames in the
        // [z][b][co][t] layout), every storing wave drains, then one lane per workgroup adds to the
        // tile's ticket; the workgroup whose add returns nsplit - 1 reads the partials with sc1
        // loads after a barrier, and resets the ticket for the next launch.
        const int Tp = (Tt + 3) & ~3;
        const auto prs = __builtin_amdgcn_make_buffer_rsrc(a.part, (short)0, (int)(CONV_SPLITK_FLOATS * 4), 0x00020000);
        const int64_t pz = (int64_t)nb * a.co_pad * Tp;  // floats per split slice
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int tb = t0 + wt + i * 16 + (lane >> 4) * 4;
                const int co = c0 + wc + j * 16 + (lane & 15);
                floatx4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float sum = acc[0][i][j][r];
#pragma unroll
                    for (int k = 1; k < NACC; ++k) sum += acc[k][i][j][r];
                    v[r] = sum;
                }
                if (tb < Tb)
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), prs,
                                                           (int)((z * pz + ((int64_t)b * a.co_pad + co) * Tp + tb) * 4), 0, 16);
            }
        __shared__ int last_arriver;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            const int tk = __hip_atomic_fetch_add(a.tickets + bx, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last_arriver = tk == nsplit - 1;
            if (tk == nsplit - 1) __hip_atomic_store(a.tickets + bx, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (!last_arriver) return;
        const int ld = a.out_ld ? a.out_ld : a.Cout;
        const int rtm = a.res_tmax ? a.res_tmax : a.Tmax;
        // thread: 4 consecutive frames of one channel
        for (int e = tid; e < (BM / 4) * BN; e += 256) {
            const int co = c0 + e / (BM / 4), tb = t0 + 4 * (e % (BM / 4));
            if (tb >= Tb || co >= a.Cout) continue;
            const int off = (int)((((int64_t)b * a.co_pad + co) * Tp + tb) * 4);
            floatx4 sum = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(prs, off, 0, 16));
            for (int zz = 1; zz < nsplit; ++zz)
                sum += __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(prs, off + (int)(zz * pz * 4), 0, 16));
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int t = tb + r;
                if (t >= Tb) break;
                float y = a.scale ? sum[r] * a.scale[co] : sum[r];
                if (a.shift) y += a.shift[co];
                if (a.act == CONV_RELU) y = fmaxf(y, 0.f);
                else if (a.act == CONV_TANH) y = tanhf(y);
                else if (a.act == CONV_SIGMOID) y = sigmoidf_(y);
                if (a.resid) y = a.resid[((int64_t)b * rtm + t) * ld + co] + y;
                a.out[((int64_t)b * a.Tmax + t) * ld + co] = y;
            }
        }
        return;
    }
    if (SPLIT) {
        // raw partial sums -> part[z][b][t][co_pad]; conv_reduce_kernel applies the epilogue
        const int64_t pb = ((int64_t)z * nb + b) * Tt;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int t = t0 + wt + i * 16 + (lane >> 4) * 4 + r;
                    const int co = c0 + wc + j * 16 + (lane & 15);
                    if (t >= Tb) continue;
                    float sum = acc[0][i][j][r];
#pragma unroll
                    for (int k = 1; k < NACC; ++k) sum += acc[k][i][j][r];
                    a.part[(pb + t) * a.co_pad + co] = sum;
                }
        return;
    }
    const int ld = a.out_ld ? a.out_ld : a.Cout;
    float* outb = a.out + (int64_t)b * a.Tmax * ld;
    const float* resb = a.resid ? a.resid + (int64_t)b * (a.res_tmax ? a.res_tmax : a.Tmax) * ld : nullptr;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int t = t0 + wt + i * 16 + (lane >> 4) * 4 + r;
                const int co = c0 + wc + j * 16 + (lane & 15);
                const bool valid = t < Tb && co < a.Cout;
                const int cc = co < a.Cout ? co : a.Cout - 1;
                float sum = acc[0][i][j][r];
#pragma unroll
                for (int k = 1; k < NACC; ++k) sum += acc[k][i][j][r];
                float y = a.scale ? sum * a.scale[cc] : sum;
                if (a.shift) y += a.shift[cc];
                if (a.act == CONV_HIGHWAY) {
                    // lanes l, l^1 hold columns 2c (H) and 2c+1 (T) of the same frame
                    const float yt = __shfl_xor(y, 1, 64);
                    if (valid && !(co & 1)) {
                        const int c = co >> 1;
                        const float hh = fmaxf(y, 0.f), tg = sigmoidf_(yt);
                        const float x = resb[(int64_t)t * ld + c];
                        outb[(int64_t)t * ld + c] = hh * tg + x * (1.f - tg);
                    }
                    continue;
                }
                if (!valid) continue;
                if (a.act == CONV_RELU) y = fmaxf(y, 0.f);
                else if (a.act == CONV_TANH) y = tanhf(y);
                else if (a.act == CONV_SIGMOID) y = sigmoidf_(y);
                if (resb) y = resb[(int64_t)t * ld + co] + y;
                outb[(int64_t)t * ld + co] = y;
            }
}

// ---------------------------------------------------------------- varlen tiles (batched KW <= 5)
// The batched Tacotron2 encoder / postnet convs (64 sentences of 60-1000 frames) as conv_kernel
// over a virtual packed frame axis: sentence b occupies T_b + 2 PAD consecutive virtual rows (its
// frames between PAD zero rows on each side), so 64-frame tiles cross sentence boundaries instead
// of padding each sentence to a tile multiple (+25 % rows at 64-frame tiles, +13 % at 32), and the
// zero rows give every output frame its own sentence's halo.  Each 64 x 64 tile reuses a weight slab
// for twice the frames of the 32-frame tiles, halving the L2 -> LDS weight stream that bounds them.
// Per output element the MFMA sequence (K steps, taps, per-tap chains summed in tap order) is
// conv_kernel's: bitwise its results.  The virtual offsets come from the device lengths (a wave
// prefix in every workgroup: the synthesis postnet runs before the host knows the step counts).
constexpr int CONV_VL_BMAX = 256;  // sentences per launch
template <int KW>
__global__ __launch_bounds__(256) void conv_vl_kernel(const ConvArgs a, int nb) {
    constexpr int PAD = (KW - 1) / 2;
    constexpr int BM = 64, WM = 2, WN = 2, BK = 16, NACC = KW;
    constexpr int BN = CONV_BN;
    constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
    constexpr int XROWS = BM + KW - 1;
    constexpr int XN = XROWS * (BK / 4);
    constexpr int WN4 = BK * KW * (BN / 4);
    constexpr int XR = (XN + 255) / 256, WR = (WN4 + 255) / 256;
    __shared__ float xs[2][XROWS][BK + 1];
    // weight slab rows padded to BNP: the B-operand read's four k-quarter lane groups (stride
    // KW * BNP floats) then fall on four disjoint 16-bank sets (KW * BNP = 16 mod 64), not one
    constexpr int BNP = BN + 16;
    static_assert((KW * BNP) % 64 == 16 || KW != 5, "bank spread for KW = 5");
    __shared__ __align__(16) float ws[2][BK][KW][BNP];
    __shared__ int vpre[CONV_VL_BMAX + 1];
    __shared__ int rowbt[XROWS];  // input row r of the tile: b << 16 | t, or -1 (a zero row)
    const int ntl = a.co_pad / BN;
    const int ntile = (int)blockIdx.x % ntl, vt = (int)blockIdx.x / ntl;
    const int c0 = ntile * BN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // ---- virtual row offsets: vpre[b] = sum_{b' < b} (T_b' + 2 PAD)
    if (wave == 0) {
        int carry = 0;
        for (int b0 = 0; b0 < nb; b0 += 64) {
            const int b = b0 + lane;
            const int len = b < nb ? (a.tmul > 1 ? a.T[b] * a.tmul : a.T[b]) + 2 * PAD : 0;
            int x = len;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int y = __shfl_up(x, d, 64);
                if (lane >= d) x += y;
            }
            if (b < nb) vpre[b + 1] = carry + x;
            carry += __shfl(x, 63, 64);
        }
        if (lane == 0) vpre[0] = 0;
    }
    __syncthreads();
    const int V0 = vt * BM;
    if (V0 >= vpre[nb]) return;  // (uniform) past the last sentence
    if (tid < XROWS) {
        const int v = V0 - PAD + tid;
        int code = -1;
        if (v >= 0 && v < vpre[nb]) {
            int lo = 0, hi = nb - 1;  // the last b with vpre[b] <= v
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (vpre[mid] <= v) lo = mid;
                else hi = mid - 1;
            }
            const int t = v - vpre[lo] - PAD;
            const int Tb = a.tmul > 1 ? a.T[lo] * a.tmul : a.T[lo];
            if (t >= 0 && t < Tb) code = (lo << 16) | t;
        }
        rowbt[tid] = code;
    }
    __syncthreads();
    const int64_t Tin = a.in_tmax ? a.in_tmax : a.Tmax;
    const int wt = (wave / WN) * (BM / WM);
    const int wc = (wave % WN) * (BN / WN);
    floatx4 acc[NACC][TM][TN];
#pragma unroll
    for (int k = 0; k < NACC; ++k)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[k][i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    // this thread's staged input rows: their source row (a valid dummy for zero rows)
    const float* xsrc[XR];
    bool xok[XR];
#pragma unroll
    for (int q = 0; q < XR; ++q) {
        const int i = min(tid + q * 256, XN - 1);
        const int code = rowbt[i / (BK / 4)];
        xok[q] = code >= 0;
        const int b = xok[q] ? code >> 16 : 0, t = xok[q] ? code & 0xFFFF : 0;
        xsrc[q] = (a.ids ? a.table + (int64_t)a.ids[(int64_t)b * a.Tmax + t] * a.Cin : a.in + ((int64_t)b * Tin + t) * a.Cin) +
                  (i % (BK / 4)) * 4;
    }
    float4 xr[XR], wr[WR];
#define VL_GLOAD(CI0)                                                                                      \
    {                                                                                                      \
        const int ci0_ = (CI0);                                                                            \
        _Pragma("unroll") for (int q = 0; q < XR; ++q) {                                                    \
            const float4 v = *reinterpret_cast<const float4*>(xsrc[q] + ci0_);                             \
            xr[q] = xok[q] ? v : float4{0.f, 0.f, 0.f, 0.f};                                               \
        }                                                                                                  \
        _Pragma("unroll") for (int q = 0; q < WR; ++q) {                                                    \
            const int i = min(tid + q * 256, WN4 - 1);                                                     \
            const int c4 = i % (BN / 4), rk = i / (BN / 4);                                                \
            wr[q] = *reinterpret_cast<const float4*>(a.W + ((int64_t)(ci0_ * KW + rk)) * a.co_pad + c0 + c4 * 4); \
        }                                                                                                  \
    }
#define VL_LSTORE(BUF)                                                                                     \
    {                                                                                                      \
        const int buf_ = (BUF);                                                                            \
        _Pragma("unroll") for (int q = 0; q < XR; ++q) {                                                    \
            const int i = tid + q * 256;                                                                   \
            if (i < XN) {                                                                                  \
                const int r = i / (BK / 4), c4 = i % (BK / 4);                                             \
                xs[buf_][r][c4 * 4 + 0] = xr[q].x;                                                         \
                xs[buf_][r][c4 * 4 + 1] = xr[q].y;                                                         \
                xs[buf_][r][c4 * 4 + 2] = xr[q].z;                                                         \
                xs[buf_][r][c4 * 4 + 3] = xr[q].w;                                                         \
            }                                                                                              \
        }                                                                                                  \
        _Pragma("unroll") for (int q = 0; q < WR; ++q) {                                                    \
            const int i = tid + q * 256;                                                                   \
            if (i < WN4) {                                                                                 \
                const int c4 = i % (BN / 4), rk = i / (BN / 4);                                            \
                *reinterpret_cast<float4*>(&ws[buf_][rk / KW][rk % KW][c4 * 4]) = wr[q];                   \
            }                                                                                              \
        }                                                                                                  \
    }
    const int nsteps = a.Cin / BK;
    VL_GLOAD(0);
    VL_LSTORE(0);
    __syncthreads();
    const int row = lane & 15, kq = lane >> 4;
    for (int st = 0; st < nsteps; ++st) {
        const int cur = st & 1;
        VL_GLOAD(min(st + 1, nsteps - 1) * BK);  // the last step reloads itself (unused)
#pragma unroll
        for (int k = 0; k < KW; ++k) {
#pragma unroll
            for (int kk = 0; kk < BK; kk += 4) {
                float av[TM], bv[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) av[i] = xs[cur][wt + i * 16 + row + k][kk + kq];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv[j] = ws[cur][kk + kq][k][wc + j * 16 + row];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[k][i][j] = mfma16x16x4(av[i], bv[j], acc[k][i][j]);
            }
        }
        VL_LSTORE(cur ^ 1);
        __syncthreads();
    }
#undef VL_GLOAD
#undef VL_LSTORE
    // epilogue (conv_kernel's): D lane l holds C[(l>>4)*4 + r][l&15]; output row lr of the tile is
    // input row lr + PAD of the map
    const int ld = a.out_ld ? a.out_ld : a.Cout;
    const int rtm = a.res_tmax ? a.res_tmax : a.Tmax;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int code = rowbt[wt + i * 16 + (lane >> 4) * 4 + r + PAD];
            if (code < 0) continue;
            const int b = code >> 16, t = code & 0xFFFF;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int co = c0 + wc + j * 16 + (lane & 15);
                if (co >= a.Cout) continue;
                float sum = acc[0][i][j][r];
#pragma unroll
                for (int k = 1; k < NACC; ++k) sum += acc[k][i][j][r];
                float y = a.scale ? sum * a.scale[co] : sum;
                if (a.shift) y += a.shift[co];
                if (a.act == CONV_RELU) y = fmaxf(y, 0.f);
                else if (a.act == CONV_TANH) y = tanhf(y);
                else if (a.act == CONV_SIGMOID) y = sigmoidf_(y);
                if (a.resid) y = a.resid[((int64_t)b * rtm + t) * ld + co] + y;
                a.out[((int64_t)b * a.Tmax + t) * ld + co] = y;
            }
        }
}

// ---------------------------------------------------------------- small-batch convolution
// The batch-1 postnet / encoder convs (T ~ 100-300 frames, ~100 output tiles) were bound by the
// tiled kernel's per-K-step global -> LDS -> barrier round trip (2 us per 16-channel step at one
// workgroup per tile, measured).  Here a workgroup owns 16 frames x 32 output channels: it stages
// its input rows (all Cin channels, KW - 1 halo rows) in LDS ONCE, then each of its CS_WAVES waves sweeps
// a slice of the K = Cin * KW reduction with the MFMA B operands (weights) loaded straight from
// the packed [Cin][KW][co_pad] layout into registers, CS_PR k-step pairs ahead, and no barrier until
// the waves' partial tiles are summed (fixed order) for the epilogue.
constexpr int CS_BM = 16, CS_BN = 32, CS_PR = 8, CS_WAVES = 8, CS_THREADS = 64 * CS_WAVES;
// TAP (Cin = 512, weights from conv_pack_frag_tap): wave w takes input channels [64 w, 64 w + 64)
// for every tap instead of a slice of the channel-major K, so a tap's 16 k-steps are one round
// whose A operands sit at compile-time offsets from one LDS address and whose weights are 8
// consecutive fragment pairs: no per-k-step index arithmetic (round 5: it was the loop's limiter,
// ~9 VALU per A operand beside the MFMAs).
constexpr int CS_TAP_CIN = 8 * CS_WAVES * CS_PR;  // 512
// N16 (TAP only, weights from conv_pack_frag_tap16): 16 output channels per workgroup, for grids
// that would leave CUs idle at 32 (the batch-1 encoder convs: 7 frame tiles x 16 channel tiles =
// 112 workgroups at L = 100).  Its accumulator chain is the 32-wide form's acc0 for the same
// channels (same MFMAs in the same order): bitwise the same outputs.
template <int KW, bool TAP, bool N16>
__global__ __launch_bounds__(CS_THREADS) void conv_small_kernel(const ConvArgs a) {
    static_assert(TAP || !N16, "the 16-channel form is tap-major only");
    constexpr int BN = N16 ? 16 : CS_BN;
    constexpr int PAD = (KW - 1) / 2;
    constexpr int XR = CS_BM + KW - 1;
    extern __shared__ float xs[];  // [XR][Cin + 1] input rows; then the waves' partial tiles
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int Tt = a.Ttile ? a.Ttile : a.Tmax;
    const int nct = a.co_pad / BN, mtiles = (Tt + CS_BM - 1) / CS_BM;
    const int ct = blockIdx.x % nct, rest = blockIdx.x / nct;
    const int b = rest / mtiles, t0 = (rest % mtiles) * CS_BM, c0 = ct * BN;
    const int Tb = a.tmul > 1 ? a.T[b] * a.tmul : a.T[b];
    if (t0 >= Tb) return;
    const int Cin = a.Cin, ldx = Cin + 1;
    const int64_t Tin = a.in_tmax ? a.in_tmax : a.Tmax;
    const int* idsb = a.ids ? a.ids + (int64_t)b * a.Tmax : nullptr;
    // B operands from the fragment-order copy Wf (conv_pack_frag): one float4 per lane per pair
    // of k-steps = W[k][c0 + r], W[k][c0 + 16 + r] at k = 8 p + q and 8 p + 4 + q; CS_PR pairs
    // in flight in a register ring (each pair's reload issued right after its MFMAs)
    const int nks = (Cin * KW) >> 2;
    const int q = lane >> 4, row = lane & 15;
    const int np = nks >> 1;  // pairs (K is a multiple of 8)
    const int p_beg = wave * np / CS_WAVES, p_end = (wave + 1) * np / CS_WAVES;
    using WT = std::conditional_t<N16, float2, float4>;
    const WT* Wf = reinterpret_cast<const WT*>(N16 ? a.Wf16 : a.Wf) + (int64_t)ct * np * 64 + lane;
    WT wr[CS_PR];
    const int pw = wave * (CS_TAP_CIN / CS_WAVES) / 8;  // (TAP: this wave's first pair of tap 0)
    if constexpr (!TAP) {
#pragma unroll
        for (int i = 0; i < CS_PR; ++i) wr[i] = Wf[(int64_t)min(p_beg + i, p_end - 1) * 64];
    } else {
#pragma unroll
        for (int i = 0; i < CS_PR; ++i) wr[i] = Wf[(int64_t)(pw + i) * 64];
    }
    {
        // every load of the stage is issued before the first LDS store (one memory round trip, beside the
        // first weight loads)
        constexpr int XPT = (XR * 128 + CS_THREADS - 1) / CS_THREADS;  // float4 per thread at Cin <= 512
        float4 xv[XPT];
#pragma unroll
        for (int u = 0; u < XPT; ++u) {
            const int i = tid + u * CS_THREADS;
            const int r = i / (Cin >> 2), c4 = i - r * (Cin >> 2), t = t0 - PAD + r;
            const bool ok = r < XR && t >= 0 && t < Tb;
            const int tc = ok ? t : 0;
            const float* src = idsb ? a.table + (int64_t)idsb[tc] * Cin : a.in + ((int64_t)b * Tin + tc) * Cin;
            const float4 v = *reinterpret_cast<const float4*>(src + 4 * (r < XR ? c4 : 0));
            xv[u] = ok ? v : float4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < XPT; ++u) {
            const int i = tid + u * CS_THREADS;
            const int r = i / (Cin >> 2), c4 = i - r * (Cin >> 2);
            if (r < XR) {
                float* d = xs + r * ldx + 4 * c4;
                d[0] = xv[u].x; d[1] = xv[u].y; d[2] = xv[u].z; d[3] = xv[u].w;
            }
        }
    }
    __syncthreads();
    // lane supplies A[row][q] = x[t0 + row + tap - PAD][ci] and B[q][n] = W[k][c0 + 16 j + n] for
    // k = 4 s + q = ci * KW + tap
    floatx4 acc0 = floatx4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    if constexpr (TAP) {
        // pairs of tap t for this wave: (t Cin + 64 w) / 8 + [0, CS_PR) (tap 0's issued before the staging)
        const float* xrow = xs + row * ldx + wave * (CS_TAP_CIN / CS_WAVES) + q;
        // (fully unrolled: a loop header would drain the weight ring's loads every tap)
#pragma unroll
        for (int tap = 0; tap < KW; ++tap) {
            float xa[2 * CS_PR];
#pragma unroll
            for (int i = 0; i < 2 * CS_PR; ++i) xa[i] = xrow[tap * ldx + 4 * i];
            const int pn = (tap + 1) * (CS_TAP_CIN / 8) + pw;
#pragma unroll
            for (int i = 0; i < CS_PR; ++i) {
                if constexpr (N16) {
                    acc0 = mfma16x16x4(xa[2 * i], wr[i].x, acc0);
                    acc0 = mfma16x16x4(xa[2 * i + 1], wr[i].y, acc0);
                } else {
                    acc0 = mfma16x16x4(xa[2 * i], wr[i].x, acc0);
                    acc1 = mfma16x16x4(xa[2 * i], wr[i].y, acc1);
                    acc0 = mfma16x16x4(xa[2 * i + 1], wr[i].z, acc0);
                    acc1 = mfma16x16x4(xa[2 * i + 1], wr[i].w, acc1);
                }
                if (tap + 1 < KW) wr[i] = Wf[(int64_t)(pn + i) * 64];
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    } else if constexpr (!N16) {
    int k0 = 8 * p_beg + q;
    int ci = k0 / KW, tap = k0 - ci * KW;
    auto next4 = [&]() {  // k += 4
        if constexpr (KW == 1) {
            ci += 4;
        } else {
            tap += 4;
#pragma unroll
            for (int w = 0; w < (4 + KW - 1) / KW; ++w) {
                const bool wrap = tap >= KW;
                tap = wrap ? tap - KW : tap;
                ci = wrap ? ci + 1 : ci;
            }
        }
    };
    auto round = [&](int pc) {
        // the round's A operands first (every LDS read in flight together), then per pair its MFMAs
        // and the reload of its ring slot, in that order (sched_barrier)
        float xa[2 * CS_PR];
#pragma unroll
        for (int i = 0; i < 2 * CS_PR; ++i) {
            xa[i] = xs[(row + tap) * ldx + min(ci, Cin - 1)];
            next4();
        }
#pragma unroll
        for (int i = 0; i < CS_PR; ++i) {
            // pairs past p_end multiply zero A operands (exact no-ops on the accumulators)
            const bool ok = pc + i < p_end;
            const float a0 = ok ? xa[2 * i] : 0.f, a1 = ok ? xa[2 * i + 1] : 0.f;
            acc0 = mfma16x16x4(a0, wr[i].x, acc0);
            acc1 = mfma16x16x4(a0, wr[i].y, acc1);
            acc0 = mfma16x16x4(a1, wr[i].z, acc0);
            acc1 = mfma16x16x4(a1, wr[i].w, acc1);
            wr[i] = Wf[(int64_t)min(pc + i + CS_PR, p_end - 1) * 64];
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    // two rounds per loop trip: the compiler drains every outstanding load at a loop header, so
    // that drain is paid once per 2 * CS_PR pairs (the second round waits only for its own slot)
    for (int pc = p_beg; pc < p_end; pc += 2 * CS_PR) {
        round(pc);
        if (pc + CS_PR < p_end) round(pc + CS_PR);
    }
    }
    __syncthreads();  // every wave is done with the input rows: reuse them for the partial tiles
    float* red = xs;  // [wave][j][lane][r]
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        red[(wave * 2 + 0) * 256 + lane * 4 + r] = acc0[r];
        red[(wave * 2 + 1) * 256 + lane * 4 + r] = acc1[r];
    }
    __syncthreads();
    const int ld = a.out_ld ? a.out_ld : a.Cout;
    const int rtm = a.res_tmax ? a.res_tmax : a.Tmax;
    for (int e = tid; e < CS_BM * BN; e += CS_THREADS) {
        const int tl = e / BN, cl = e % BN, t = t0 + tl, co = c0 + cl;
        if (t >= Tb || co >= a.Cout) continue;
        const int j = cl >> 4, src_lane = (tl >> 2) * 16 + (cl & 15), idx = src_lane * 4 + (tl & 3);
        float sum = red[j * 256 + idx];  // the waves' partial tiles in wave order
#pragma unroll
        for (int w = 1; w < CS_WAVES; ++w) sum += red[(2 * w + j) * 256 + idx];
        float y = a.scale ? sum * a.scale[co] : sum;
        if (a.shift) y += a.shift[co];
        if (a.act == CONV_RELU) y = fmaxf(y, 0.f);
        else if (a.act == CONV_TANH) y = tanhf(y);
        else if (a.act == CONV_SIGMOID) y = sigmoidf_(y);
        if (a.resid) y = a.resid[((int64_t)b * rtm + t) * ld + co] + y;
        a.out[((int64_t)b * a.Tmax + t) * ld + co] = y;
    }
}

template <int KW>
bool launch_small(const ConvArgs& a, int B, int frames_hint, hipStream_t s, hipError_t* err) {
    static const int limit = getenv("TTS_CONV_SMALL") ? atoi(getenv("TTS_CONV_SMALL")) : 1024;  // frames; 0 = off
    if (!a.Wf || frames_hint > limit || a.pool2 || a.act == CONV_HIGHWAY || (a.Cin & 3) || a.Cin > 512 ||
        (a.co_pad % CS_BN) || ((a.Cin * KW) & 7))
        return false;
    const int Tt = a.Ttile ? a.Ttile : a.Tmax;
    const size_t smem = sizeof(float) * std::max((size_t)(CS_BM + KW - 1) * (a.Cin + 1), (size_t)2 * 256 * CS_WAVES);
    const int tiles = ((Tt + CS_BM - 1) / CS_BM) * B;
    const dim3 grid(tiles * (a.co_pad / CS_BN));
    // 16-channel tiles while the 32-channel grid leaves CUs idle (TTS_CONV_N16: that grid bound)
    static const int n16_max = getenv("TTS_CONV_N16") ? atoi(getenv("TTS_CONV_N16")) : 128;
    if (a.wf_tap && a.Cin == CS_TAP_CIN && a.Wf16 && (int)grid.x <= n16_max)
        hipLaunchKernelGGL((conv_small_kernel<KW, true, true>), dim3(tiles * (a.co_pad / 16)), dim3(CS_THREADS), smem, s, a);
    else if (a.wf_tap && a.Cin == CS_TAP_CIN)
        hipLaunchKernelGGL((conv_small_kernel<KW, true, false>), grid, dim3(CS_THREADS), smem, s, a);
    else if (a.wf_tap)
        return false;  // (tap-major weights for another Cin: never packed so, conv_pack_frag_tap refuses)
    else
        hipLaunchKernelGGL((conv_small_kernel<KW, false, false>), grid, dim3(CS_THREADS), smem, s, a);
    *err = hipGetLastError();
    return true;
}

__global__ void conv_pack_kernel(const float* W, int Cout, int Cin, int KW, int co_pad, float* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)Cin * KW * co_pad;
    if (i >= total) return;
    const int co = i % co_pad;
    const int k = (i / co_pad) % KW;
    const int ci = i / ((int64_t)co_pad * KW);
    out[i] = co < Cout ? W[((int64_t)co * Cin + ci) * KW + k] : 0.f;
}

// packed [K][co_pad] -> fragment order [co_pad / 32][K / 8][64 lanes][4]: lane (q, r) of pair p
// holds W[8p + q][32ct + r], W[8p + q][32ct + 16 + r], W[8p + 4 + q][32ct + r], W[8p + 4 + q][32ct + 16 + r]
__global__ void conv_pack_frag_kernel(const float* W, int K, int co_pad, float* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)K * co_pad) return;
    const int e = i & 3, lane = (i >> 2) & 63;
    const int64_t rest = i >> 8;
    const int np = K >> 3;
    const int p = rest % np, ct = rest / np;
    const int q = lane >> 4, r = lane & 15;
    const int k = 8 * p + 4 * (e >> 1) + q, co = 32 * ct + 16 * (e & 1) + r;
    out[i] = W[(int64_t)k * co_pad + co];
}

// packed [Cin * KW][co_pad] (k = ci KW + tap) -> the tap-major fragment order of conv_small_kernel's
// TAP form: k' = tap Cin + ci, then as conv_pack_frag over k'
__global__ void conv_pack_frag_tap_kernel(const float* W, int Cin, int KW, int co_pad, float* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int K = Cin * KW;
    if (i >= (int64_t)K * co_pad) return;
    const int e = i & 3, lane = (i >> 2) & 63;
    const int64_t rest = i >> 8;
    const int np = K >> 3;
    const int p = rest % np, ct = rest / np;
    const int q = lane >> 4, r = lane & 15;
    const int kt = 8 * p + 4 * (e >> 1) + q, co = 32 * ct + 16 * (e & 1) + r;
    const int tap = kt / Cin, ci = kt - tap * Cin;
    out[i] = W[(int64_t)(ci * KW + tap) * co_pad + co];
}

// the same tap-major order for 16-column tiles: [co_pad / 16][K / 8][64 lanes][2], lane (q, r) of
// pair p holding W[8p + q][16ct + r], W[8p + 4 + q][16ct + r] (k' = tap Cin + ci)
__global__ void conv_pack_frag_tap16_kernel(const float* W, int Cin, int KW, int co_pad, float* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int K = Cin * KW;
    if (i >= (int64_t)K * co_pad) return;
    const int e = i & 1, lane = (i >> 1) & 63;
    const int64_t rest = i >> 7;
    const int np = K >> 3;
    const int p = rest % np, ct = rest / np;
    const int q = lane >> 4, r = lane & 15;
    const int kt = 8 * p + 4 * e + q, co = 16 * ct + r;
    const int tap = kt / Cin, ci = kt - tap * Cin;
    out[i] = W[(int64_t)(ci * KW + tap) * co_pad + co];
}

__global__ void conv_pack_bank_kernel(const float* W, int Cout, int Cin, int k, int KWmax, int co_off, int co_pad,
                                      float* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)Cin * k * Cout) return;
    const int co = i % Cout;
    const int j = (i / Cout) % k;
    const int ci = i / ((int64_t)Cout * k);
    const int slot = j + (KWmax - 1) / 2 - (k - 1) / 2;
    out[((int64_t)ci * KWmax + slot) * co_pad + co_off + co] = W[((int64_t)co * Cin + ci) * k + j];
}

__global__ void linear_pack_kernel(const float* W, int Cout, int Cin, int co_offset, int stride, int co_pad,
                                   float* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)Cin * Cout) return;
    const int n = i % Cout, ci = i / Cout;
    out[(int64_t)ci * co_pad + co_offset + (int64_t)n * stride] = W[(int64_t)n * Cin + ci];
}

__global__ void copy_strided_kernel(const float* src, int n, float* dst, int stride) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[(int64_t)i * stride] = src[i];
}

__global__ void fold_bn_kernel(const float* bias, const float* gamma, const float* beta, const float* mean,
                               const float* var, int C, float eps, float* scale, float* shift) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float sc = gamma[c] / sqrtf(var[c] + eps);
    scale[c] = sc;
    shift[c] = beta[c] + ((bias ? bias[c] : 0.f) - mean[c]) * sc;
}

// Split-K epilogue: out[b][t][co] = act(scale * sum_z part[z][b][t][co] + shift) (+ resid), the
// partials summed in split order.  Rows t >= T_b are left untouched (as the one-pass epilogue).
__global__ void conv_reduce_kernel(const ConvArgs a, int B, int nsplit) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int Tt = a.Ttile ? a.Ttile : a.Tmax;
    const int64_t total = (int64_t)B * Tt * a.Cout;
    if (i >= total) return;
    const int co = i % a.Cout;
    const int t = (i / a.Cout) % Tt;
    const int b = i / ((int64_t)a.Cout * Tt);
    if (t >= (a.tmul > 1 ? a.T[b] * a.tmul : a.T[b])) return;
    float sum = 0.f;
    for (int z = 0; z < nsplit; ++z) sum += a.part[(((int64_t)z * B + b) * Tt + t) * a.co_pad + co];
    float y = a.scale ? sum * a.scale[co] : sum;
    if (a.shift) y += a.shift[co];
    if (a.act == CONV_RELU) y = fmaxf(y, 0.f);
    else if (a.act == CONV_TANH) y = tanhf(y);
    else if (a.act == CONV_SIGMOID) y = sigmoidf_(y);
    const int ld = a.out_ld ? a.out_ld : a.Cout;
    if (a.resid) y = a.resid[((int64_t)b * (a.res_tmax ? a.res_tmax : a.Tmax) + t) * ld + co] + y;
    a.out[((int64_t)b * a.Tmax + t) * ld + co] = y;
}

template <int KW>
hipError_t launch_kw(const ConvArgs& a, int B, int frames_hint, hipStream_t s) {
    const dim3 block(256);
    if constexpr (KW == 1 || KW == 5) {
        hipError_t e = hipSuccess;
        if (launch_small<KW>(a, B, frames_hint, s, &e)) return e;
    }
    constexpr int BK = KW <= 5 ? 16 : (KW <= 8 ? 8 : 4);
    const int Tt = a.Ttile ? a.Ttile : a.Tmax;
    const int tiles = ((Tt + 15) / 16) * (a.co_pad / CONV_BN) * B;
    if (a.part && a.act != CONV_HIGHWAY && tiles < 256) {
        // split the K steps so that the launch fills the chip: nsplit x tiles <= 1024
        const int nsteps = a.Cin / BK;
        int ns = 1;
        static const int ns_max = getenv("TTS_CONV_NSMAX") ? atoi(getenv("TTS_CONV_NSMAX")) : 16;  // A/B knob
        while (ns * 2 <= ns_max && tiles * ns * 2 <= 1024 && nsteps % (ns * 2) == 0 && nsteps / (ns * 2) >= 2) ns *= 2;
        if (ns > 1 && (size_t)ns * B * ((Tt + 3) & ~3) * a.co_pad <= CONV_SPLITK_FLOATS) {
            // TTS_CONV_FUSED_REDUCE=1: the reduction rides in the same launch (last-arriving
            // workgroup per tile); measured slower than the separate reduce launch at batch 1
            // (34.5 vs 23.3 + 7.4 us per layer), so off by default
            static const bool fused_ok = getenv("TTS_CONV_FUSED_REDUCE") && getenv("TTS_CONV_FUSED_REDUCE")[0] == '1';
            ConvArgs b = a;
            if (!fused_ok || tiles > CONV_TICKETS) b.tickets = nullptr;
            hipLaunchKernelGGL((conv_kernel<KW, 16, 1, 4, true>), dim3(tiles * ns), block, 0, s, b, ns, B);
            if (!b.tickets) {
                const int64_t total = (int64_t)B * Tt * a.Cout;
                hipLaunchKernelGGL(conv_reduce_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a, B, ns);
            }
            return hipGetLastError();
        }
    }
    const char* vle = getenv("TTS_CONV_VL");  // A/B + test knob (read per launch: one per layer)
    const bool vl_off = vle && vle[0] == '0';
    if (KW == 5 && frames_hint > 4096 && !vl_off && !a.pool2 && a.act != CONV_HIGHWAY && B <= CONV_VL_BMAX &&
        Tt < 65536 - 4 && B * (Tt + 4) < (1 << 30) / 64) {
        const int vtiles = (B * (Tt + 2 * ((KW - 1) / 2)) + 63) / 64;  // upper bound: tiles past the end exit
        hipLaunchKernelGGL(conv_vl_kernel<5>, dim3((unsigned)(vtiles * (a.co_pad / CONV_BN))), block, 0, s, a, B);
        return hipGetLastError();
    }
    if (frames_hint <= 4096) {
        const dim3 grid(((Tt + 15) / 16) * (a.co_pad / CONV_BN) * B);
        hipLaunchKernelGGL((conv_kernel<KW, 16, 1, 4>), grid, block, 0, s, a);
    } else if (KW == 5) {
        // the Tacotron2 encoder / postnet convs (sentences of 60-1000 frames): 32-frame tiles halve
        // the last tile's padding rows; measured -0.3 ms per configs[2] batch (the KW 1 / 3 / 8 / 16
        // CBHG launches of configs[4] measured slower with them and keep 64)
        const dim3 grid(((Tt + 31) / 32) * (a.co_pad / CONV_BN) * B);
        hipLaunchKernelGGL((conv_kernel<KW, 32, 2, 2>), grid, block, 0, s, a);
    } else {
        const dim3 grid(((Tt + 63) / 64) * (a.co_pad / CONV_BN) * B);
        hipLaunchKernelGGL((conv_kernel<KW, 64, 2, 2>), grid, block, 0, s, a);
    }
    return hipGetLastError();
}

}  // namespace

hipError_t conv_pack(const float* W, int Cout, int Cin, int KW, float* out, hipStream_t s) {
    const int co_pad = conv_co_pad(Cout);
    const int64_t total = (int64_t)Cin * KW * co_pad;
    hipLaunchKernelGGL(conv_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, s, W, Cout, Cin, KW, co_pad, out);
    return hipGetLastError();
}

hipError_t conv_pack_frag(const float* W, int K, int co_pad, float* out, hipStream_t s) {
    if ((K & 7) || (co_pad % CS_BN)) return hipErrorInvalidValue;
    const int64_t total = (int64_t)K * co_pad;
    hipLaunchKernelGGL(conv_pack_frag_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, W, K, co_pad, out);
    return hipGetLastError();
}

hipError_t conv_pack_frag_tap(const float* W, int Cin, int KW, int co_pad, float* out, hipStream_t s) {
    if (Cin != CS_TAP_CIN || (co_pad % CS_BN)) return hipErrorInvalidValue;
    const int64_t total = (int64_t)Cin * KW * co_pad;
    hipLaunchKernelGGL(conv_pack_frag_tap_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, W, Cin, KW, co_pad,
                       out);
    return hipGetLastError();
}
hipError_t conv_pack_frag_tap16(const float* W, int Cin, int KW, int co_pad, float* out, hipStream_t s) {
    if (Cin != CS_TAP_CIN || (co_pad % CS_BN)) return hipErrorInvalidValue;
    const int64_t total = (int64_t)Cin * KW * co_pad;
    hipLaunchKernelGGL(conv_pack_frag_tap16_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, W, Cin, KW,
                       co_pad, out);
    return hipGetLastError();
}
bool conv_frag_tap_ok(int Cin) { return Cin == CS_TAP_CIN; }

hipError_t conv_pack_bank(const float* W, int Cout, int Cin, int k, int KWmax, int co_off, int co_pad, float* out,
                          hipStream_t s) {
    if (k < 1 || k > KWmax) return hipErrorInvalidValue;
    const int64_t total = (int64_t)Cin * k * Cout;
    hipLaunchKernelGGL(conv_pack_bank_kernel, dim3((total + 255) / 256), dim3(256), 0, s, W, Cout, Cin, k, KWmax, co_off,
                       co_pad, out);
    return hipGetLastError();
}

hipError_t linear_pack_strided(const float* W, int Cout, int Cin, int co_offset, int stride, int co_pad, float* out,
                               hipStream_t s) {
    const int64_t total = (int64_t)Cin * Cout;
    hipLaunchKernelGGL(linear_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, s, W, Cout, Cin, co_offset, stride,
                       co_pad, out);
    return hipGetLastError();
}

hipError_t linear_pack_as_conv(const float* W, int Cout, int Cin, int co_offset, int co_pad, float* out,
                               hipStream_t s) {
    return linear_pack_strided(W, Cout, Cin, co_offset, 1, co_pad, out, s);
}

hipError_t copy_strided(const float* src, int n, float* dst, int stride, hipStream_t s) {
    hipLaunchKernelGGL(copy_strided_kernel, dim3((n + 255) / 256), dim3(256), 0, s, src, n, dst, stride);
    return hipGetLastError();
}

hipError_t fold_bn(const float* bias, const float* gamma, const float* beta, const float* mean, const float* var,
                   int C, float eps, float* scale, float* shift, hipStream_t s) {
    hipLaunchKernelGGL(fold_bn_kernel, dim3((C + 255) / 256), dim3(256), 0, s, bias, gamma, beta, mean, var, C, eps,
                       scale, shift);
    return hipGetLastError();
}

hipError_t conv_launch(const ConvArgs& a, int KW, int B, int frames_hint, hipStream_t s) {
    const int bk = KW <= 5 ? 16 : (KW <= 8 ? 8 : 4);
    if (a.Cin % bk || (a.act == CONV_HIGHWAY && (a.Cout & 1))) return hipErrorInvalidValue;
    switch (KW) {
        case 1: return launch_kw<1>(a, B, frames_hint, s);
        case 3: return launch_kw<3>(a, B, frames_hint, s);
        case 5: return launch_kw<5>(a, B, frames_hint, s);
        case 8: return launch_kw<8>(a, B, frames_hint, s);
        case 16: return launch_kw<16>(a, B, frames_hint, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace tts

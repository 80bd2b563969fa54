// Batched Griffin-Lim vocoder (AudioProcessor.inv_mel_spectrogram / inv_spectrogram,
// utils/audio.py:154-201, librosa 0.6.2 stft/istft semantics) for gfx950.
//
// Precision follows the reference exactly where it is observable: the magnitude |S|^power and
// every FFT are float64 (scipy.fftpack on float64 frames), the STFT matrix is rounded to
// complex64 before the phase is taken (librosa stft's dtype), and the overlap-added signal y is
// float32 (librosa istft's dtype), accumulated frame by frame in float32 as librosa does.  GL
// amplifies rounding ~100x over 60 iterations, so this is what keeps the waveform within 1e-4.
//
// HBM layout (per call):
//   S      [B][Fmax][1025] f32    |S|^power, frame-major (one 4.1 KB row per frame; computed in
//                                 float64, stored rounded: the linear path's values are float32
//                                 already, the mel path's rounding moves the waveform ~1e-6)
//   frames [2][B][Fmax][WINP]     windowed inverse-FFT output of every frame, window support only
//                                 (WIN = 1102 samples; the padded Hann is zero elsewhere).  The
//                                 batched (unfused) loop stores them float32, rounded once before
//                                 librosa's float32 overlap-add (round 3: float64 slots were 2/3 of
//                                 its HBM traffic); the fused and persistent loops, which gather
//                                 every sample from its <= 5 contributing frames, keep float64 (their
//                                 sc1 4-byte gathers measured 2.4 -> 4.3 us per iteration)
// One workgroup per (sentence, frame) per iteration does the whole GL iteration for its frame:
//   overlap-add gather of the previous iteration's frames (<= 5 contributors per sample) with the
//   window-sum-square normalisation and the STFT's reflect padding -> window -> 2048-point real
//   FFT (1024-point complex Stockham radix-4 in LDS) -> S * X/|X| -> inverse real FFT -> window
//   -> store the frame.  Iterations ping-pong the frames buffer (a frame's neighbours still read
//   the previous iteration), one launch per iteration, replayed from a hipGraph.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <tuple>
#include <type_traits>
#include <vector>

#include "common.h"

#ifndef GLP_SLEEP
#define GLP_SLEEP 1  // persistent loop: s_sleep between neighbour-tag polls
#endif

using namespace tts;

namespace {

typedef float spec_t;    // |S|^power storage
typedef float frame_t;   // windowed iSTFT frame storage (every loop: rounded once before librosa's
                         // float32 overlap-add, which adds each float64 frame into a float32 signal)
// the persistent loop's frame storage: one 8-byte granule per sample, {tag : 32 | float32 sample},
// the tag naming the iteration that wrote it (round 4; replaces float64 slots + per-frame flags)
struct gran_t {
    unsigned long long v;
};
__device__ __forceinline__ double fval(float x) { return (double)x; }
__device__ __forceinline__ double fval(gran_t x) { return (double)__uint_as_float((unsigned)x.v); }
__device__ __forceinline__ void fstore(float* p, double v, unsigned) { *p = (float)v; }
__device__ __forceinline__ void fstore(gran_t* p, double v, unsigned tag) {
    p->v = ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint((float)v);
}

constexpr int NFFT = 2048;
constexpr int NB = 1025;  // bins
constexpr int NH = 1024;  // complex FFT size
constexpr int GL_THREADS = 256;
constexpr int MAG_KT = 64;  // magnitude kernel tile: bins (one per lane) ...
constexpr int MAG_FT = 16;  // ... x frames (MAG_FT / 4 per wave)
constexpr int SCAN_THREADS = 1024;
constexpr int SCAN_PER = 8;  // samples per thread per scan tile
constexpr int SCAN_CHUNK = 4096;  // de-emphasis output samples per workgroup

struct Geo {
    int hop, win, woff, winp;  // woff = (NFFT - win) / 2, winp = win + (woff - fb) rounded up to 4
    int fb;                    // a frame slot holds samples [fb, fb + winp): fb = woff rounded down to
                               // even, so sample pairs (2n, 2n+1) are 16-byte aligned
};

struct GLConst {
    const double* win;    // [2048] padded periodic Hann
    const double* win2;   // [2048] win^2
    const double2* tw;    // [2048] e^{-2 pi i m / 2048}
};

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return double2{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
__device__ __forceinline__ double2 cconj(double2 a) { return double2{a.x, -a.y}; }

// Per-thread twiddles of the four twiddled Stockham passes (Ns = 4, 16, 64, 256): loaded once per
// kernel with the other operands, so the FFT passes wait only on LDS.
struct FftTw {
    double2 w[4][3];
};
__device__ __forceinline__ FftTw load_fft_tw(const double2* __restrict__ tw) {
    FftTw t;
    const int j = threadIdx.x;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int Ns = 4 << (2 * p);
        const int k = j & (Ns - 1);
#pragma unroll
        for (int r = 1; r < 4; ++r) t.w[p][r - 1] = tw[k * r * (512 / Ns)];
    }
    return t;
}

// Stockham radix-4, 5 passes, 256 threads x 1 butterfly.  Returns the buffer holding the result.
template <bool INV>
__device__ double2* fft1024(double2* src, double2* dst, const FftTw& tw) {
    const int j = threadIdx.x;
#pragma unroll
    for (int Ns = 1, p = -1; Ns < NH; Ns *= 4, ++p) {
        const int k = j & (Ns - 1);
        double2 v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = src[j + r * 256];
        if (Ns > 1) {
#pragma unroll
            for (int r = 1; r < 4; ++r) {
                double2 w = tw.w[p][r - 1];
                if (INV) w = cconj(w);
                v[r] = cmul(v[r], w);
            }
        }
        const double2 a0 = double2{v[0].x + v[2].x, v[0].y + v[2].y};
        const double2 a1 = double2{v[0].x - v[2].x, v[0].y - v[2].y};
        const double2 a2 = double2{v[1].x + v[3].x, v[1].y + v[3].y};
        const double2 a3 = double2{v[1].x - v[3].x, v[1].y - v[3].y};
        // -i*a3 = (a3.y, -a3.x); +i*a3 = (-a3.y, a3.x)
        const double2 m3 = INV ? double2{-a3.y, a3.x} : double2{a3.y, -a3.x};
        const int idxD = (j / Ns) * Ns * 4 + k;
        dst[idxD] = double2{a0.x + a2.x, a0.y + a2.y};
        dst[idxD + Ns] = double2{a1.x + m3.x, a1.y + m3.y};
        dst[idxD + 2 * Ns] = double2{a0.x - a2.x, a0.y - a2.y};
        dst[idxD + 3 * Ns] = double2{a1.x - m3.x, a1.y - m3.y};
        __syncthreads();
        double2* t = src;
        src = dst;
        dst = t;
    }
    return src;
}

// LDS slot of complex point i in the fft1024_regs buffers: rows of 16 points (256 B, all 64
// banks) with the 16-byte columns XOR-swizzled by 5 * (row mod 4).  The Ns = 1 pass stores lane
// j's points at 4j + r (16 lanes span 4 rows, columns {0, 4, 8, 12}) and the Ns = 4 pass at
// 16 (j/4) + j%4 + 4r (4 rows, columns {0..3}): both land on 16 distinct columns instead of
// 4-way bank conflicts; contiguous reads stay a permutation of one row.
__device__ __forceinline__ int swz(int i) { return i ^ (5 * ((i >> 4) & 3)); }

// ---- two-level 1024-point complex FFT of one 256-thread workgroup (round 5).  1024 = 4 x 256:
// one radix-4 step ACROSS the four waves, thread-local in registers, and one 256-point Stockham
// radix-4 FFT per wave whose three LDS exchanges stay inside that wave's own 256-slot region.  A
// wave's LDS operations execute in issue order, so the wave-local exchanges need no barrier: the
// transform has ONE workgroup barrier (the cross-wave hand-over) instead of four.
//   layout A (thread t = 64 w + l):  v[r] = z[t + 256 r]          (edge_sample: STFT input, iSTFT output)
//   layout B (wave w, lane l):        v[r] = Z[4 (l + 64 r) + w]   (the spectrum's bins)
// Forward, decimation in frequency, A -> B:
//   u_q[m] = W1024^(m q) sum_s z[m + 256 s] W4^(s q)  (thread m: a butterfly over its registers),
//   Z[4 k1 + q] = sum_m u_q[m] W256^(m k1)            (wave q: 256-point FFT over m = l + 64 r);
// inverse, decimation in time, B -> A: the same two steps in reverse order with conjugate twiddles.
// Region q of a buffer is slots [256 q, 256 q + 256), points XOR-swizzled by swz (the Stockham
// store patterns of a 256-point pass are the first three of the 1024-point one).
// threadIdx.x through an opaque copy: LDS addresses derived from it are recomputed per transform
// instead of hoisted out of the persistent loop, where dozens of them would stay live (and spill)
__device__ __forceinline__ int tid_opaque() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}
template <bool INV>
__device__ __forceinline__ void bfly4(double2 (&v)[4]) {
    const double2 a0 = double2{v[0].x + v[2].x, v[0].y + v[2].y};
    const double2 a1 = double2{v[0].x - v[2].x, v[0].y - v[2].y};
    const double2 a2 = double2{v[1].x + v[3].x, v[1].y + v[3].y};
    const double2 a3 = double2{v[1].x - v[3].x, v[1].y - v[3].y};
    // -i*a3 = (a3.y, -a3.x); +i*a3 = (-a3.y, a3.x)
    const double2 m3 = INV ? double2{-a3.y, a3.x} : double2{a3.y, -a3.x};
    v[0] = double2{a0.x + a2.x, a0.y + a2.y};
    v[1] = double2{a1.x + m3.x, a1.y + m3.y};
    v[2] = double2{a0.x - a2.x, a0.y - a2.y};
    v[3] = double2{a1.x - m3.x, a1.y - m3.y};
}
// Twiddles of the two-level FFT (entries of the 2048-point table tw[m] = W2048^m):
//   fx(q)     = W1024^(t q), q = 1..3            (forward cross-wave step, thread t)
//   ix(r)     = W1024^((l + 64 r) w)             (inverse cross-wave step, wave w, lane l)
//   ps(p, r)  = W_(4 Ns)^(r (l mod Ns)), r = 1..3 (wave pass p = 0, 1, 2: Ns = 4, 16, 64)
// TwRegs holds all 16 in registers for the kernel's lifetime (the persistent loop: one wave per
// SIMD, registers to spare); TwTable reads the L2-resident table where they are used (the
// register-budget forms).  Same values either way, so the forms are bitwise equal.
struct TwRegs {
    double2 f[3], i[4], p[3][3];
    __device__ __forceinline__ void load(const double2* __restrict__ tw) {
        const int t = threadIdx.x, l = t & 63, w = t >> 6;
#pragma unroll
        for (int q = 1; q < 4; ++q) f[q - 1] = tw[2 * t * q];
#pragma unroll
        for (int r = 0; r < 4; ++r) i[r] = tw[2 * (l + 64 * r) * w];
#pragma unroll
        for (int ps = 0; ps < 3; ++ps) {
            const int Ns = 4 << (2 * ps);
#pragma unroll
            for (int r = 1; r < 4; ++r) p[ps][r - 1] = tw[(l & (Ns - 1)) * r * (512 / Ns)];
        }
    }
    __device__ __forceinline__ double2 tw_at(int) const { return double2{0.0, 0.0}; }  // (TwTable only)
    __device__ __forceinline__ double2 fx(int q) const { return f[q - 1]; }
    __device__ __forceinline__ double2 ix(int r) const { return i[r]; }
    __device__ __forceinline__ double2 ps(int p_, int r) const { return p[p_][r - 1]; }
};
// TwMix (the two-per-CU persistent form's register budget): the forward cross-wave twiddles in
// registers, the wave passes' from a 252-entry LDS copy (pt: [pass][l mod Ns][r - 1], 4 KB), the
// inverse cross-wave ones from the table (fetched ahead of the wave FFT).
constexpr int TW_LDS = 3 * (4 + 16 + 64);
__device__ __forceinline__ int tw_lds_base(int p_) { return p_ == 0 ? 0 : p_ == 1 ? 12 : 60; }
typedef __attribute__((address_space(1))) const double g_d;  // global
typedef __attribute__((address_space(3))) const double l_d;  // LDS
struct TwMix {
    g_d* tw;  // (address-space-qualified scalars: the table reads stay global / LDS loads)
    l_d* pt;
    double2 f[3];
    __device__ __forceinline__ void load(const double2* __restrict__ t) {
        const int j = threadIdx.x;
        tw = (g_d*)t;
#pragma unroll
        for (int q = 1; q < 4; ++q) f[q - 1] = t[2 * j * q];
    }
    // fill the LDS copy (every thread; the caller's barrier orders it before the first use)
    __device__ __forceinline__ static void fill(double2* lds, const double2* __restrict__ t) {
        for (int e = threadIdx.x; e < TW_LDS; e += blockDim.x) {
            const int p_ = e < 12 ? 0 : e < 60 ? 1 : 2, o = e - tw_lds_base(p_);
            const int Ns = 4 << (2 * p_), k = o / 3, r = o % 3 + 1;
            lds[e] = t[k * r * (512 / Ns)];
        }
    }
    __device__ __forceinline__ double2 tw_at(int k) const { return double2{tw[2 * k], tw[2 * k + 1]}; }
    __device__ __forceinline__ double2 fx(int q) const { return f[q - 1]; }
    __device__ __forceinline__ double2 ix(int r) const {
        return tw_at(2 * (((int)threadIdx.x & 63) + 64 * r) * ((int)threadIdx.x >> 6));
    }
    __device__ __forceinline__ double2 ps(int p_, int r) const {
        const int Ns = 4 << (2 * p_), e = tw_lds_base(p_) + ((int)threadIdx.x & (Ns - 1)) * 3 + r - 1;
        return double2{pt[2 * e], pt[2 * e + 1]};
    }
};
struct TwTable {
    const double2* __restrict__ tw;
    __device__ __forceinline__ double2 tw_at(int k) const { return tw[k]; }
    __device__ __forceinline__ double2 fx(int q) const { return tw[2 * (int)threadIdx.x * q]; }
    __device__ __forceinline__ double2 ix(int r) const {
        return tw[2 * (((int)threadIdx.x & 63) + 64 * r) * ((int)threadIdx.x >> 6)];
    }
    __device__ __forceinline__ double2 ps(int p_, int r) const {
        const int Ns = 4 << (2 * p_);
        return tw[((int)threadIdx.x & (Ns - 1)) * r * (512 / Ns)];
    }
};

// 256-point Stockham radix-4 FFT of one wave, in place in its region rg: enters with v[r] =
// u[l + 64 r] (the first pass's operands, so it reads no LDS), leaves v[r] = U[l + 64 r] (the last
// pass's outputs stay in registers).  Each pass's twiddles are fetched one pass ahead.
template <bool INV, class TW>
__device__ __forceinline__ void wave_fft256(double2 (&v)[4], double2* rg, int l, const TW& tw) {
    asm volatile("" : "+v"(l));
    double2 w[3];
#pragma unroll
    for (int r = 1; r < 4; ++r) w[r - 1] = tw.ps(0, r);
#pragma unroll
    for (int p = -1; p < 3; ++p) {
        const int Ns = 1 << (2 * (p + 1));
        if (p >= 0) {
            double2 wn[3];
            if (p < 2) {
#pragma unroll
                for (int r = 1; r < 4; ++r) wn[r - 1] = tw.ps(p + 1, r);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = rg[swz(l + 64 * r)];
#pragma unroll
            for (int r = 1; r < 4; ++r) v[r] = cmul(v[r], INV ? cconj(w[r - 1]) : w[r - 1]);
            if (p < 2) {
#pragma unroll
                for (int r = 0; r < 3; ++r) w[r] = wn[r];
            }
        }
        bfly4<INV>(v);
        if (p == 2) return;  // Ns = 64: lane l's outputs are U[l + 64 r]
        const int idxD = (l / Ns) * Ns * 4 + (l & (Ns - 1));
#pragma unroll
        for (int r = 0; r < 4; ++r) rg[swz(idxD + r * Ns)] = v[r];
        __builtin_amdgcn_wave_barrier();  // (code motion only: the wave's LDS ops run in order)
    }
}
// Forward two-level FFT, layout A -> B.  Writes every region of wr (the caller's earlier readers
// of wr must be past a barrier); one barrier.
template <class TW>
__device__ __forceinline__ void fft2l_fwd(double2 (&v)[4], double2* wr, const TW& tw) {
    const int t = tid_opaque(), l = t & 63, w = threadIdx.x >> 6;
    bfly4<false>(v);
#pragma unroll
    for (int q = 1; q < 4; ++q) v[q] = cmul(v[q], tw.fx(q));
#pragma unroll
    for (int q = 0; q < 4; ++q) wr[256 * q + swz(t)] = v[q];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = wr[256 * w + swz(l + 64 * r)];
    wave_fft256<false>(v, wr + 256 * w, l, tw);
}
// Inverse two-level FFT, layout B -> A (unnormalised).  Uses region w of wr first (the caller's
// earlier readers of that region must be past a barrier), then reads every region; one barrier.
template <class TW>
__device__ __forceinline__ void fft2l_inv(double2 (&v)[4], double2* wr, const TW& tw) {
    const int t = tid_opaque(), l = t & 63, w = threadIdx.x >> 6;
    double2* rg = wr + 256 * w;
    double2 iw[4];  // (fetched ahead of the wave FFT: in flight during it when read from the table)
#pragma unroll
    for (int r = 0; r < 4; ++r) iw[r] = tw.ix(r);
    wave_fft256<true>(v, rg, l, tw);
    if (w != 0) {  // (wave 0's twiddles are 1)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = cmul(v[r], cconj(iw[r]));
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) rg[swz(l + 64 * r)] = v[r];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = wr[256 * q + swz(t)];
    bfly4<true>(v);
}

// Bin k of the thread's register r in layout B
__device__ __forceinline__ int bin2l(int t, int r) { return 4 * ((t & 63) + 64 * r) + (t >> 6); }
__device__ __forceinline__ int bin2l(int r) { return bin2l((int)threadIdx.x, r); }
// STFT value of bin k from zk = Z[k mod 1024] and zm = Z[(1024 - k) mod 1024] (real-FFT split),
// rounded to complex64 (librosa stft dtype), then |S| exp(i angle X) (angle(0) = 0) in float64
// (utils/audio.py:187-188) by one reciprocal square root (the float-rounded components square
// exactly in double): no divisions on the iteration's critical path.  Im = 0 at DC and Nyquist
// (istft: .real of the Hermitian extension).
__device__ __forceinline__ double2 spec_bin(double2 zk, double2 zm, double2 t, double s, bool edge) {
    const double2 zc = cconj(zm);
    const double2 E = double2{0.5 * (zk.x + zc.x), 0.5 * (zk.y + zc.y)};
    const double2 O = double2{0.5 * (zk.y - zc.y), -0.5 * (zk.x - zc.x)};  // -i (zk - zc) / 2
    const double xre = (double)(float)(E.x + (t.x * O.x - t.y * O.y));
    const double xim = (double)(float)(E.y + (t.x * O.y + t.y * O.x));
    const double m2 = xre * xre + xim * xim;
    // the hardware reciprocal square root (~2^-23) and one Newton step (~2^-45): the reference's
    // unit phase is itself complex64 (np.exp(1j * np.angle(X)) on a complex64 X)
    double ri = __builtin_amdgcn_rsq(m2);
    ri = fma(0.5 * ri, fma(-m2 * ri, ri, 1.0), ri);
    double2 xv = m2 > 0.0 ? double2{s * (xre * ri), s * (xim * ri)} : double2{s, 0.0};
    if (edge) xv.y = 0.0;
    return xv;
}
// Forward spectrum step in layout B: v = Z on entry, X = |S| X/|X| on return; the Nyquist bin
// X[1024] goes to xnyq of thread 0 (wave 0, lane 0: it holds Z[0] and is the only reader of
// X[1024]).  zb: 1024 slots (one barrier after the Z stores; the caller's earlier readers of zb
// must be past a barrier).  tk(r) = W2048^k and sk(r) = |S|[k] for the thread's bins k = bin2l(r);
// tnyq / snyq: the same for k = 1024 (thread 0).
template <class TK, class SK>
__device__ __forceinline__ void spectrum2l(double2 (&v)[4], double2* zb, TK tk, SK sk, double2 tnyq, double snyq,
                                           double2& xnyq) {
    const int t = tid_opaque();
#pragma unroll
    for (int r = 0; r < 4; ++r) zb[swz(bin2l(t, r))] = v[r];
    __syncthreads();
    if (threadIdx.x == 0) xnyq = spec_bin(v[0], v[0], tnyq, snyq, true);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int k = bin2l(t, r);
        v[r] = spec_bin(v[r], zb[swz((NH - k) & (NH - 1))], tk(r), sk(r), k == 0);
    }
}
// Inverse real-FFT pre-split in layout B: v = X on entry, z'[k] = E + i O on return
// (E = (X[k] + conj X[N-k]) / 2, O = (X[k] - conj X[N-k]) / 2 * conj(t)); xb: 1024 slots (one
// barrier after the X stores; the caller's earlier readers of xb must be past a barrier).
template <class TK>
__device__ __forceinline__ void presplit2l(double2 (&v)[4], double2* xb, TK tk, double2 xnyq) {
    const int t = tid_opaque();
#pragma unroll
    for (int r = 0; r < 4; ++r) xb[swz(bin2l(t, r))] = v[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int k = bin2l(t, r);
        const double2 xk = v[r];
        double2 xm = xb[swz((NH - k) & (NH - 1))];
        if (r == 0 && k == 0) xm = xnyq;  // (bin 0 pairs with the Nyquist bin: thread 0, register 0)
        const double2 xc = cconj(xm);
        const double2 E = double2{0.5 * (xk.x + xc.x), 0.5 * (xk.y + xc.y)};
        const double2 D = double2{0.5 * (xk.x - xc.x), 0.5 * (xk.y - xc.y)};
        const double2 O = cmul(D, cconj(tk(r)));
        v[r] = double2{E.x - O.y, E.y + O.x};  // E + i O
    }
}

// Real sample i (0..7) of thread j in layout A (fft2l_fwd's input, fft2l_inv's output): complex point j + 256 (i/2),
// real part (i even) or imaginary part (i odd) = real sample 2 j + 512 (i/2) + (i & 1).
__device__ __forceinline__ int edge_sample(int j, int i) { return 2 * j + 512 * (i >> 1) + (i & 1); }

// Bijective XCD-aware remap: consecutive logical frames share an XCD (their OLA gathers
// re-read each other's frames through that XCD's L2).  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int n) {
    const int q = n >> 3, r = n & 7, x = bid & 7, i = bid >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// np.pad(..., mode='reflect') index map for a signal of length N (any overhang).
__device__ __forceinline__ int reflect_idx(int p, int N) {
    if ((unsigned)p < (unsigned)N) return p;  // interior: no division
    if (N == 1) return 0;
    const int period = 2 * (N - 1);
    int pp = p % period;
    if (pp < 0) pp += period;
    return pp < N ? pp : period - pp;
}

// float32 y[p] of the previous iteration's iSTFT (librosa istft): float64 frame contributions
// added frame by frame into a float32 accumulator, divided (float32) by the float32 window
// sum-square where it exceeds float32 tiny.  q = p + n_fft/2 is the untrimmed position.
template <typename FT>
__device__ __forceinline__ float ola_sample(const FT* __restrict__ fr, int q, int F, const Geo& g,
                                            const double* __restrict__ win2) {
    if (q < g.woff) return 0.f;
    int ilo = q - g.woff - g.win + 1;
    ilo = ilo <= 0 ? 0 : (ilo + g.hop - 1) / g.hop;
    int ihi = (q - g.woff) / g.hop;
    if (ihi > F - 1) ihi = F - 1;
    float y = 0.f, wss = 0.f;
    for (int i = ilo; i <= ihi; ++i) {
        const int o = q - i * g.hop;  // offset inside frame i (0..2047)
        y = (float)((double)y + fval(fr[(int64_t)i * g.winp + (o - g.fb)]));
        wss = (float)((double)wss + win2[o]);
    }
    return wss > 1.17549435e-38f ? y / wss : y;
}

// ola_sample with the <= OLA_MAX contributing frames' loads issued together (the sum still runs
// frame by frame in index order; absent contributors add exact zeros): bitwise equal to it.
constexpr int OLA_MAX = 5;  // ceil(win / hop) for the reference geometry (1102 / 275)
template <typename FT>
__device__ __forceinline__ float ola_sample_unrolled(const FT* __restrict__ fr, int q, int F, const Geo& g,
                                                     const double* __restrict__ win2) {
    if (q < g.woff) return 0.f;
    int ilo = q - g.woff - g.win + 1;
    ilo = ilo <= 0 ? 0 : (ilo + g.hop - 1) / g.hop;
    int ihi = (q - g.woff) / g.hop;
    if (ihi > F - 1) ihi = F - 1;
    double fv[OLA_MAX], wv[OLA_MAX];
#pragma unroll
    for (int k = 0; k < OLA_MAX; ++k) {
        const int i = ilo + k;
        const int o = q - i * g.hop;
        const bool ok = i <= ihi;
        fv[k] = ok ? fval(fr[(int64_t)i * g.winp + (o - g.fb)]) : 0.0;
        wv[k] = ok ? win2[o] : 0.0;
    }
    float y = 0.f, wss = 0.f;
#pragma unroll
    for (int k = 0; k < OLA_MAX; ++k) {
        y = (float)((double)y + fv[k]);
        wss = (float)((double)wss + wv[k]);
    }
    return wss > 1.17549435e-38f ? y / wss : y;
}

// ---------------------------------------------------------------- |S|^power
struct MagArgs {
    int mode;  // TTS_GL_FROM_MEL / TTS_GL_FROM_LINEAR
    const float* spec;
    int n_in, Fmax;
    const int* F;
    const double* pinv;  // [n_mels][1025]: pinv(mel basis) transposed (lanes read consecutive bins)
    spec_t* S;
    float min_db, ref_db, power, max_norm;
    int signal_norm, symmetric, clip;
};

// _denormalize (utils/audio.py:96-112) then the exponent of _db_to_amp(x + ref_level_db)
// (:125-126), in float32 as numpy computes them on the float32 network output.
__device__ __forceinline__ float denorm_db(float x, const MagArgs& a) {
    float d = x;
    if (a.signal_norm) {
        if (a.symmetric) {
            if (a.clip) d = fminf(fmaxf(d, -a.max_norm), a.max_norm);
            d = ((d + a.max_norm) * -a.min_db / (2.f * a.max_norm)) + a.min_db;
        } else {
            if (a.clip) d = fminf(fmaxf(d, 0.f), a.max_norm);
            d = (d * -a.min_db / a.max_norm) + a.min_db;
        }
    }
    return (d + a.ref_db) * 0.05f;
}
// the amplitude 10^e: powf (the mel path: 80 values per frame) or exp10f (the linear path: 1025)
__device__ __forceinline__ float denorm_to_amp(float x, const MagArgs& a) { return powf(10.f, denorm_db(x, a)); }
__device__ __forceinline__ float amp_of_db(float x, const MagArgs& a) { return exp10f(denorm_db(x, a)); }

// inv_spectrogram's |S|: S (float32) ** power in float32, then widened (utils/audio.py:156-160).
// The two float32 steps as numpy has them, each within an ulp or two of its powf: the amplitude
// 10^e by exp10f, and power 1.5 (the reference configs) as a * sqrt(a).  A streaming launch with
// no LDS, LIN_PER elements per thread (round 4's tile launch with two powf per bin: 788 us at
// configs[4], dispatch- and VALU-bound).
constexpr int LIN_PER = 16;
__global__ __launch_bounds__(256) void gl_linear_magnitude_kernel(const MagArgs a) {
    const int b = blockIdx.y;
    const int64_t n = (int64_t)a.F[b] * NB;  // the sentence's frames < F[b], each a 1025-bin row
    const int64_t base = (int64_t)blockIdx.x * (256 * LIN_PER) + threadIdx.x;
    if (base >= n) return;
    const float* sp = a.spec + (int64_t)b * a.Fmax * NB;
    spec_t* S = a.S + (int64_t)b * a.Fmax * NB;
    float x[LIN_PER];
#pragma unroll
    for (int i = 0; i < LIN_PER; ++i) {
        const int64_t e = base + i * 256;
        x[i] = e < n ? sp[e] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < LIN_PER; ++i) {
        const int64_t e = base + i * 256;
        const float amp = amp_of_db(x[i], a);
        if (e < n) S[e] = (spec_t)(a.power == 1.5f ? amp * sqrtf(amp) : powf(amp, a.power));
    }
}

// Tile = MAG_KT bins x MAG_FT frames per workgroup: the pinv columns of the tile's bins staged in
// LDS once, the frames' amplitudes (float, as numpy has them) computed into LDS, then lane = bin,
// each wave MAG_FT / 4 frames, every (bin, frame) dot product summed over mels in order.
__global__ __launch_bounds__(256) void gl_magnitude_kernel(const MagArgs a) {
    const int b = blockIdx.z;
    const int Fb = a.F[b];
    const int f0 = blockIdx.y * MAG_FT;
    if (f0 >= Fb) return;
    const int nf = min(MAG_FT, Fb - f0);
    const float* sp = a.spec + ((int64_t)b * a.Fmax + f0) * a.n_in;
    spec_t* S = a.S + ((int64_t)b * a.Fmax + f0) * NB;
    const int tid = threadIdx.x;
    const int k0 = blockIdx.x * MAG_KT;
    __shared__ double pw[80][MAG_KT];
    __shared__ float amp[MAG_FT][80];
    // fixed trip counts (n_in <= 80): every staging load of the tile is in flight at once
    constexpr int PWL = 80 * MAG_KT / 256, AML = MAG_FT * 80 / 256;
    double pv[PWL];
    float sv[AML];
#pragma unroll
    for (int j = 0; j < PWL; ++j) {
        const int i = tid + j * 256, m = i / MAG_KT, kk = i % MAG_KT;
        pv[j] = m < a.n_in && k0 + kk < NB ? a.pinv[(int64_t)m * NB + k0 + kk] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < AML; ++j) {
        const int i = tid + j * 256, f = i / 80, m = i % 80;
        sv[j] = f < nf && m < a.n_in ? sp[f * a.n_in + m] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < PWL; ++j) {
        const int i = tid + j * 256;
        pw[i / MAG_KT][i % MAG_KT] = pv[j];
    }
#pragma unroll
    for (int j = 0; j < AML; ++j) {
        const int i = tid + j * 256, f = i / 80, m = i % 80;
        amp[f][m] = f < nf && m < a.n_in ? denorm_to_amp(sv[j], a) : 0.f;
    }
    __syncthreads();
    // _mel_to_linear: max(1e-10, pinv(M) . S) in float64 (utils/audio.py:64-66), then ** power
    const int lane = tid & 63, wave = tid >> 6, k = k0 + lane;
    constexpr int FW = MAG_FT / 4;
    double acc[FW];
#pragma unroll
    for (int i = 0; i < FW; ++i) acc[i] = 0.0;
    // a fixed trip count (n_in <= 80: the staged rows past n_in are zeros, whose products add +0.0)
    // keeps the LDS reads in flight ahead of the FMAs
#pragma unroll 8
    for (int m = 0; m < 80; ++m) {
        const double w = pw[m][lane];
#pragma unroll
        for (int i = 0; i < FW; ++i) acc[i] += w * (double)amp[wave * FW + i][m];
    }
    if (k < NB) {
#pragma unroll
        for (int i = 0; i < FW; ++i) {
            const int f = wave * FW + i;
            if (f < nf) {
                // power 1.5 (the reference configs): x * sqrt(x), within an ulp of pow in float64
                // and far below the float32 rounding of the stored value; else pow
                const double x = fmax(acc[i], 1e-10);
                S[(int64_t)f * NB + k] = (spec_t)(a.power == 1.5f ? x * sqrt(x) : pow(x, (double)a.power));
            }
        }
    }
}

// ---------------------------------------------------------------- GL iteration
struct IterArgs {
    const spec_t* S;      // [B][Fmax][1025]
    const float* y;       // [B][Nmax] the previous iteration's float32 signal (gl_ola_kernel)
    const void* prev;     // FUSED: the previous iteration's frames (overlap-added here instead)
    int64_t Nmax;
    void* next;           // frames written by this iteration (frame_t; gran_t for the initial iSTFT of the persistent loop)
    const int* F;
    int Fmax;
    int B;
    Geo g;
    GLConst c;
    const double* phase_u;  // initial iSTFT only: [B][1025][Fmax] or null (device RNG)
    unsigned long long seed;
    unsigned* zero_flags;   // initial iSTFT only: the persistent loop's tag words to clear, or null
    int* zero_status;       // ... and its status word
    const double2* wt;      // gl_iter_wave_kernel: [16][4] pass-2 twiddles
    const double2* winc;    // gl_iter_wave_kernel: [4][64] window cosine seeds (see tts_gl_create)
    double wrot;            // ... and the recurrence factor 2 cos(2 pi 128 / win)
    unsigned gtag;          // initial iSTFT into granules (gran_t): the tag of iteration 0
};

__device__ __forceinline__ double hash_uniform(unsigned long long seed, unsigned long long idx) {
    unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (idx + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

// FUSED (small batches): the frame's own 2048 STFT input samples are overlap-added from the
// previous iteration's frames inside this launch (bitwise the values gl_ola_kernel would store),
// so an iteration is one launch instead of two.
template <bool INIT, bool FUSED, typename FT>
// Four workgroups per CU (32 KB of LDS, <= 128 VGPRs each).  Measured at B = 64: the same speed
// as three workgroups with the FFT twiddles held in registers, faster than five (which spill).
__global__ __launch_bounds__(GL_THREADS, 4) void gl_iter_kernel(const IterArgs a) {
    const int b = blockIdx.y;
    const int f = xcd_remap(blockIdx.x, gridDim.x);
    const int Fb = a.F[b];
    // the persistent loop's status word is cleared by block (0, 0) even when the run is empty
    // (a speculative batch-1 run whose frame count was clamped to 0): its final overlap-add launch
    // copies the word to the host, which must not see an earlier run's failure
    if (INIT && a.zero_status && threadIdx.x == 0 && (blockIdx.x | blockIdx.y) == 0) *a.zero_status = 0;
    if (f >= Fb) return;
    const Geo g = a.g;
    const int tid = threadIdx.x;
    if (INIT && tid == 0 && a.zero_flags)  // the persistent loop that follows reads tags of frames < F[b] only
        a.zero_flags[(int64_t)b * a.Fmax + f] = 0u;
    __shared__ __align__(16) double2 buf0[NH];  // forward wave regions, then the spectrum X
    __shared__ __align__(16) double2 buf1[NH];  // Z, then the inverse wave regions
    // (the Nyquist bin X[1024] stays in a register of thread 0, its only writer and reader)
    double2 xnyq = double2{0.0, 0.0};
    const TwTable twt{a.c.tw};
    const spec_t* Sf = a.S + ((int64_t)b * a.Fmax + f) * NB;
    // ---- phase 0: the frame's global operands are issued before anything waits: window, |S|,
    // the input samples (the FFT and split twiddles, an L2-resident table, are read where used:
    // holding them across the forward FFT would cost a wave per SIMD)
    constexpr int PN = NFFT / GL_THREADS;  // samples per thread (8)
    // |S| of the thread's bins k = bin2l(r) (layout B), and of the Nyquist bin on thread 0
    double sk[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) sk[r] = (double)Sf[bin2l(r)];
    const double snyq = tid == 0 ? (double)Sf[NH] : 0.0;
    // the padded Hann at this thread's samples: the analysis window of the STFT input (the
    // forward FFT's layout-A registers) and the synthesis window of the iSTFT output (the inverse
    // FFT's, layout A again) sit at the same sample indices
    double wo[PN];
#pragma unroll
    for (int i = 0; i < PN; ++i) {
        const int m = edge_sample(tid, i), n = m - g.woff;
        wo[i] = n >= 0 && n < g.win ? a.c.win[m] : 0.0;
    }
    double2 v[4];
    if (!INIT) {
        // ---- STFT frame f of the previous iteration's float32 signal (librosa stft, centre reflect pad)
        const int N = g.hop * (Fb - 1);
        const float* yb = a.y + (int64_t)b * a.Nmax;
        float yi[PN];
#pragma unroll
        for (int i = 0; i < PN; ++i) {
            const int n = edge_sample(tid, i);  // the forward FFT's operands stay in registers
            const bool sup = n >= g.woff && n < g.woff + g.win;  // the padded Hann's support
            if (FUSED) {
                const FT* fb = static_cast<const FT*>(a.prev) + (int64_t)b * a.Fmax * g.winp;
                yi[i] = sup ? ola_sample_unrolled(fb, reflect_idx(f * g.hop + n - NFFT / 2, N) + NFFT / 2, Fb, g, a.c.win2)
                            : 0.f;
            } else {
                yi[i] = sup ? yb[reflect_idx(f * g.hop + n - NFFT / 2, N)] : 0.f;
            }
        }
        // z[n] = x[2n] + i x[2n+1] == real x[0..2047]
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = double2{wo[2 * r] * (double)yi[2 * r], wo[2 * r + 1] * (double)yi[2 * r + 1]};
        fft2l_fwd(v, buf0, twt);
        spectrum2l(v, buf1, [&](int r) { return a.c.tw[bin2l(r)]; }, [&](int r) { return sk[r]; }, a.c.tw[NH], snyq,
                   xnyq);
    } else {
        // ---- initial phases exp(2 pi i U), U ~ U[0,1)  (utils/audio.py:183), per bin of layout B
        auto init_bin = [&](int k, double sv) {
            const double u = a.phase_u ? a.phase_u[((int64_t)b * NB + k) * a.Fmax + f]
                                       : hash_uniform(a.seed, ((unsigned long long)b * NB + k) * 1048576ull + f);
            double sn, cs;
            sincospi(2.0 * u, &sn, &cs);  // (exp(2 pi i u) without rounding 2 pi u first)
            return double2{sv * cs, (k == 0 || k == NB - 1) ? 0.0 : sv * sn};
        };
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = init_bin(bin2l(r), sk[r]);
        if (tid == 0) xnyq = init_bin(NH, snyq);
    }
    // ---- inverse real FFT (istft: ifft of the Hermitian-extended spectrum, .real => Im X_0 =
    // Im X_N/2 = 0, set where X is formed)
    presplit2l(v, buf0, [&](int r) { return a.c.tw[bin2l(r)]; }, xnyq);
    fft2l_inv(v, buf1, twt);
    // ---- window and store the support [woff, woff+win) in float64 (ytmp of librosa istft), from
    // the inverse FFT's registers
    FT* out = static_cast<FT*>(a.next) + ((int64_t)b * a.Fmax + f) * g.winp;
#pragma unroll
    for (int i = 0; i < PN; ++i) {
        const int n = edge_sample(tid, i) - g.woff;
        const double zv = (i & 1) ? v[i >> 1].y : v[i >> 1].x;
        if (n >= 0 && n < g.win) fstore(out + (n + g.woff - g.fb), wo[i] * (zv * (1.0 / NH)), a.gtag);
    }
}

// ---------------------------------------------------------------- GL iteration, one wave per frame
// The batched form of gl_iter_kernel<false, false> (same inputs: the previous iteration's float32
// signal; same output: the windowed float64 frame), with each frame's whole iteration on ONE
// wave: the 1024-point complex FFT as radix 16 x 16 x 4 with 16 points per lane in registers and
// two wave-local LDS transposes per FFT, so no pass waits on a workgroup barrier and every
// butterfly's operands stay in VGPRs.  Index map (lane L, register r):
//   pass 1:  z[L + 64 r]                     radix-16 over r, x W1024^(L k2)
//   pass 2:  lane p1 + 4 k2, register p2     radix-16 over p2, x W64^(p1 q2)
//   pass 3:  lane r3 + 4 k2, register 4j+p1  radix-4 over p1
//   output:  lane r3 + 4 k2, register 4j+q1 holds Z[256 q1 + 64 j + 16 r3 + k2]
// The real-FFT split, the phase step and the inverse pre-split run per bin pair (k, 1024 - k) in
// the lane that owns k in the pass-1 layout of the inverse FFT; the partner's pre-split value moves
// to its owner lane (64 - L) through LDS.  LDS slots are XOR-swizzled so every exchange is free of
// bank conflicts (ds_write_b128 8-lane groups, ds_read_b128 16-lane groups).
// Twiddles: wt[k2][L] = W1024^(L k2) and wt[16 + q2][L] = W64^((L & 3) q2) (host-built, f64).
constexpr int WV_SLOTS = NH + 1;  // LDS complex slots per wave (the Nyquist bin at slot 1024)

// W32^m = e^{-i pi m / 16}, m < 8 (the split twiddle steps of the bin-pair loop)
__device__ constexpr double kW32[8][2] = {
    {1.00000000000000000000, -0.00000000000000000000},
    {0.98078528040323043058, -0.19509032201612824808},
    {0.92387953251128673848, -0.38268343236508978178},
    {0.83146961230254523567, -0.55557023301960217765},
    {0.70710678118654757274, -0.70710678118654746172},
    {0.55557023301960228867, -0.83146961230254523567},
    {0.38268343236508983729, -0.92387953251128673848},
    {0.19509032201612833135, -0.98078528040323043058}};

__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return double2{a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return double2{a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ double2 cmulf(double2 a, double2 w) {  // a * w
    return double2{fma(a.x, w.x, -(a.y * w.y)), fma(a.x, w.y, a.y * w.x)};
}
__device__ __forceinline__ double2 cmulcf(double2 a, double2 w) {  // a * conj(w)
    return double2{fma(a.x, w.x, a.y * w.y), fma(a.y, w.x, -(a.x * w.y))};
}
template <bool INV>
__device__ __forceinline__ double2 rotq(double2 a) {  // a * (-i) forward, a * (+i) inverse
    return INV ? double2{-a.y, a.x} : double2{a.y, -a.x};
}
template <bool INV>
__device__ __forceinline__ void dft4(double2& a0, double2& a1, double2& a2, double2& a3) {
    const double2 t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3), t3 = rotq<INV>(csub(a1, a3));
    a0 = cadd(t0, t2);
    a1 = cadd(t1, t3);
    a2 = csub(t0, t2);
    a3 = csub(t1, t3);
}
// a * W16^E (E in 1..9; the inverse uses conj(W16^E))
template <int E, bool INV>
__device__ __forceinline__ double2 tw16(double2 a) {
    constexpr double C1 = 0.92387953251128675613, S1 = 0.38268343236508977173, C2 = 0.70710678118654752440;
    if constexpr (E == 4) return rotq<INV>(a);
    if constexpr (E == 2) {  // (1 - i) / sqrt 2
        return INV ? double2{C2 * (a.x - a.y), C2 * (a.x + a.y)} : double2{C2 * (a.x + a.y), C2 * (a.y - a.x)};
    }
    if constexpr (E == 6) {  // (-1 - i) / sqrt 2
        return INV ? double2{-C2 * (a.x + a.y), C2 * (a.x - a.y)} : double2{C2 * (a.y - a.x), -C2 * (a.x + a.y)};
    }
    constexpr double wr = E == 1 ? C1 : E == 3 ? S1 : -C1;  // E = 1, 3, 9
    constexpr double wi = E == 1 ? -S1 : E == 3 ? -C1 : S1;
    return INV ? cmulcf(a, double2{wr, wi}) : cmulf(a, double2{wr, wi});
}
// in-register 16-point DFT: v[n] -> v[k] (natural order), as 4 x 4 with W16 twiddles
template <bool INV>
__device__ __forceinline__ void dft16(double2 (&v)[16]) {
#pragma unroll
    for (int n1 = 0; n1 < 4; ++n1) dft4<INV>(v[n1], v[n1 + 4], v[n1 + 8], v[n1 + 12]);  // k2 at v[n1 + 4 k2]
    v[5] = tw16<1, INV>(v[5]);
    v[9] = tw16<2, INV>(v[9]);
    v[13] = tw16<3, INV>(v[13]);
    v[6] = tw16<2, INV>(v[6]);
    v[10] = tw16<4, INV>(v[10]);
    v[14] = tw16<6, INV>(v[14]);
    v[7] = tw16<3, INV>(v[7]);
    v[11] = tw16<6, INV>(v[11]);
    v[15] = tw16<9, INV>(v[15]);
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) dft4<INV>(v[4 * k2], v[4 * k2 + 1], v[4 * k2 + 2], v[4 * k2 + 3]);  // X[4 k1 + k2] at v[4 k2 + k1]
    double2 o[16];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) o[4 * k1 + k2] = v[4 * k2 + k1];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = o[i];
}
// LDS slots (8-byte words; every exchange moves real parts, then imaginary parts, through one
// 1025-word buffer).  Bank rules: ds_write_b64 in 16-lane contiguous groups over 32 banks,
// ds_read_b64 in 32-lane halves over 64 banks; these swizzles keep every exchange conflict-free.
__device__ __forceinline__ int wv_a1(int k2, int n1) { return k2 * 64 + (n1 ^ (4 * (k2 & 7))); }
__device__ __forceinline__ int wv_a2(int k2, int p1, int q2) { return k2 * 64 + 4 * (q2 ^ (k2 & 7)) + (p1 ^ (k2 & 3)); }
__device__ __forceinline__ int wv_sig(int k) { return k ^ (((k >> 4) & 3) << 2); }

// All-to-all of one wave's 16 complex registers through `lds`: real parts, then imaginary parts.
// Each round overwrites only registers whose value has already been stored (the real parts are
// read back into the real halves after every lane stored them), so 8 KB of LDS suffice.
template <class WS, class RS>
__device__ __forceinline__ void wave_xchg(double2 (&v)[16], double* lds, WS wslot, RS rslot) {
#pragma unroll
    for (int r = 0; r < 16; ++r) lds[wslot(r)] = v[r].x;
    __syncthreads();  // one wave per workgroup: orders the lanes' LDS writes before the reads
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r].x = lds[rslot(r)];
    __syncthreads();  // the imaginary stores below do not depend on these reads
#pragma unroll
    for (int r = 0; r < 16; ++r) lds[wslot(r)] = v[r].y;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r].y = lds[rslot(r)];
}

// 1024-point complex FFT of one wave (forward: e^{-i}, inverse: e^{+i}, unnormalised).
// In: v[r] = z[L + 64 r].  Out: v[4 j + q1] = Z[256 q1 + 64 j + 16 (L & 3) + (L >> 2)].
// Twiddles: pass 1 multiplies register k2 by w^k2, w = W1024^L (one load), the powers built by a
// product tree (depth <= 4, a few ulp); pass 2 reads W64^(p1 q2) from the wave's 64-entry LDS
// table t2[q2][p1] (4 distinct addresses per read).  The vector-memory path was the bound.
// Ends after a barrier that follows the last LDS reads.
template <bool INV>
__device__ __forceinline__ void wave_fft1024(double2 (&v)[16], double* lds, const double2* t2, __amdgpu_buffer_rsrc_t tw,
                                             int lane) {
    // the lane index is laundered per call: otherwise the inverse FFT reuses the forward's loads
    // and LDS addresses, which then stay live (and spill) across the spectrum step
    int L = lane;
    asm volatile("" : "+v"(L));
    const double2 w1 = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(tw, 32 * L, 0, 0));
    dft16<INV>(v);
    {
        auto mul = [&](double2 a, double2 w) { return INV ? cmulcf(a, w) : cmulf(a, w); };
        const double2 w2 = cmulf(w1, w1), w4 = cmulf(w2, w2), w8 = cmulf(w4, w4);
        const double2 w3 = cmulf(w2, w1), w12 = cmulf(w8, w4);
        v[1] = mul(v[1], w1);
        v[2] = mul(v[2], w2);
        v[3] = mul(v[3], w3);
        v[4] = mul(v[4], w4);
        v[5] = mul(v[5], cmulf(w4, w1));
        v[6] = mul(v[6], cmulf(w4, w2));
        v[7] = mul(v[7], cmulf(w4, w3));
        v[8] = mul(v[8], w8);
        v[9] = mul(v[9], cmulf(w8, w1));
        v[10] = mul(v[10], cmulf(w8, w2));
        v[11] = mul(v[11], cmulf(w8, w3));
        v[12] = mul(v[12], w12);
        v[13] = mul(v[13], cmulf(w12, w1));
        v[14] = mul(v[14], cmulf(w12, w2));
        v[15] = mul(v[15], cmulf(w12, w3));
    }
    const int p1 = L & 3, K2 = L >> 2;
    wave_xchg(v, lds, [&](int k2) { return wv_a1(k2, L); }, [&](int p2) { return wv_a1(K2, p1 + 4 * p2); });
    dft16<INV>(v);
#pragma unroll
    for (int q2 = 1; q2 < 16; ++q2) {
        const double2 w = t2[q2 * 4 + p1];
        v[q2] = INV ? cmulcf(v[q2], w) : cmulf(v[q2], w);
    }
    __syncthreads();  // the previous exchange's last reads are done before this one's stores
    wave_xchg(v, lds, [&](int q2) { return wv_a2(K2, p1, q2); },
              [&](int r) { return wv_a2(K2, r & 3, 4 * (r >> 2) + p1); });
#pragma unroll
    for (int j = 0; j < 4; ++j) dft4<INV>(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
    __syncthreads();
}

// STFT value X (rounded to complex64, librosa stft dtype) -> |S| X / |X| (angle(0) = 0).  The
// reference's unit phase is itself complex64 (np.exp(1j * np.angle(X)) on a complex64 X), so the
// hardware reciprocal square root plus one Newton step (relative error far below float32's) is
// ample; X may carry any power-of-two scale (the result does not).  |X|^2 of two floats is
// within fp64 range, so no operand scaling is needed.
__device__ __forceinline__ double2 unit_phase(double2 X, double s) {
    const double xre = (double)(float)X.x, xim = (double)(float)X.y;
    const double m2 = fma(xre, xre, xim * xim);
    double r = __builtin_amdgcn_rsq(m2);
    r = fma(0.5 * r, fma(-m2 * r, r, 1.0), r);
    const double sr = s * r;  // (|S| folded into the reciprocal: one product per component)
    return m2 > 0.0 ? double2{xre * sr, xim * sr} : double2{s, 0.0};
}
// inverse real-FFT pre-split, times 2: z'[k] = E + i O, 2E = X[k] + conj X[N-k],
// 2O = (X[k] - conj X[N-k]) * conj(t) (the factor 1/2 is folded into the output scale)
__device__ __forceinline__ double2 inv_presplit2(double2 xk, double2 xm, double2 t) {
    const double2 E = double2{xk.x + xm.x, xk.y - xm.y};
    const double2 D = double2{xk.x - xm.x, xk.y + xm.y};
    const double2 O = cmulcf(D, t);
    return double2{E.x - O.y, E.y + O.x};
}

// buffer-resource access (SGPR base + 32-bit lane offset; out-of-range loads read 0, stores drop)
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float buf_f32(__amdgpu_buffer_rsrc_t r, int voff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, 0));
}
__device__ __forceinline__ float buf_f32s(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ double buf_f64(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
__device__ __forceinline__ double2 buf_c64(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ void buf_st_f64(double v, __amdgpu_buffer_rsrc_t r, int voff) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, voff, 0, 0);
}

// INIT: the initial iSTFT of exp(2 pi i U) |S| (utils/audio.py:183) on the same wave layout: no
// STFT, the bin pairs' X formed from the phases, then the inverse half as below (the batched
// loops' first launch; the 256-thread gl_iter_kernel<true> took ~1.5x a wave iteration).
template <bool INIT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 4))) void gl_iter_wave_kernel(const IterArgs a) {
    const int b = blockIdx.y;
    const int f = xcd_remap(blockIdx.x, gridDim.x);
    const int Fb = a.F[b];
    if (f >= Fb) return;
    const Geo g = a.g;
    const int L = threadIdx.x;
    __shared__ double lds[WV_SLOTS];
    __shared__ double2 t2[64];  // W64^(p1 q2) at [q2][p1]
    const auto rS = buf_rsrc(a.S + ((int64_t)b * a.Fmax + f) * NB, NB * 4);
    const auto rC = buf_rsrc(a.winc, 4 * 64 * 16);
    const auto rT = buf_rsrc(a.c.tw, NFFT * 16);
    const auto rP = buf_rsrc(a.wt, 64 * 16);
    // ---- STFT input: z[L + 64 r] = x[2 (L + 64 r)] + i x[2 (L + 64 r) + 1], x = window * y_pad.
    // The periodic Hann at sample s is 1/2 - 1/2 c(s), c(s) = cos(2 pi (s - woff) / win); the lane's
    // samples step by 128 per register, so c follows the Chebyshev recurrence
    // c_{r+1} = 2 cos(theta) c_r - c_{r-1} (one fma per sample from two seeds per parity, a few
    // ulp over 16 steps, instead of 16 window-table loads).  Outside the support the sample is
    // exactly 0: the support-sized y range reads 0 there, or (reflected frames) a select.
    const double K = a.wrot;
    double2 v[16];
    const int r3 = L & 3, K2 = L >> 2;
    const int zb = wv_sig(L);                         // Z[L + 64 m]
    const int mb = wv_sig((64 - L) & 63) + (L == 0 ? 64 : 0);
    double zkr[8], zmr[8], z512r = 0.0, z512i = 0.0;
    t2[L] = buf_c64(rP, 16 * L, 0);  // first LDS use: ordered before the reads by the FFT's barriers
    if constexpr (!INIT) {
        const int N = g.hop * (Fb - 1);
        const int base = f * g.hop - NFFT / 2;
        float y0[16], y1[16];
        const bool interior = base + g.woff >= 0 && base + g.woff + g.win <= N;
        if (interior) {  // the support needs no reflection
            const auto rY = buf_rsrc(a.y + (int64_t)b * a.Nmax + base + g.woff, (unsigned)g.win * 4);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int s = 2 * (L + 64 * r) - g.woff;
                y0[r] = buf_f32(rY, s * 4);
                y1[r] = buf_f32(rY, (s + 1) * 4);
            }
        } else {
            const auto rY = buf_rsrc(a.y + (int64_t)b * a.Nmax, (unsigned)N * 4);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int s = 2 * (L + 64 * r);
                const bool i0 = s >= g.woff && s < g.woff + g.win, i1 = s + 1 >= g.woff && s + 1 < g.woff + g.win;
                y0[r] = i0 ? buf_f32(rY, reflect_idx(base + s, N) * 4) : 0.f;
                y1[r] = i1 ? buf_f32(rY, reflect_idx(base + s + 1, N) * 4) : 0.f;
            }
        }
        {
            const double2 s0 = buf_c64(rC, 16 * L, 0), s1 = buf_c64(rC, 16 * L, 1024);  // (c_0, c_1) per parity
            double a0 = s0.x, a1 = s0.y, b0 = s1.x, b1 = s1.y;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                v[r] = double2{fma(-0.5, a0, 0.5) * (double)y0[r], fma(-0.5, b0, 0.5) * (double)y1[r]};
                const double a2 = fma(K, a1, -a0), b2 = fma(K, b1, -b0);
                a0 = a1;
                a1 = a2;
                b0 = b1;
                b1 = b2;
            }
        }
        wave_fft1024<false>(v, lds, t2, rT, L);
        // ---- Z to LDS in natural (swizzled) order, real parts then imaginary parts; bin pairs
        // (k, 1024 - k), k = L + 64 m, m < 8, plus k = 512.  sig() only permutes bits 2-3 by bits 4-5,
        // so every address below is one per-lane base plus a multiple of 64 slots: Z[k] at zb + 64 m,
        // Z[1024 - k] at mb + 64 (15 - m) (for lane 0, m = 0 that is the spare slot 1024: Z[0] is taken
        // from its own Z[k] read, and the partner store that pair does not have lands there).  Every
        // LDS store is unconditional: a divergent store makes the compiler branch around the partner's
        // computation and spill.
        const int wb = wv_sig(16 * r3 + K2);              // this lane's output Z[256 q1 + 64 j + wb']
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q1 = 0; q1 < 4; ++q1) lds[wb + 256 * q1 + 64 * j] = v[4 * j + q1].x;
        __syncthreads();
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            zkr[m] = lds[zb + 64 * m];
            zmr[m] = lds[mb + 64 * (15 - m)];
        }
        if (L == 0) zmr[0] = zkr[0];
        z512r = lds[512];  // sig(512) = 512
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q1 = 0; q1 < 4; ++q1) lds[wb + 256 * q1 + 64 * j] = v[4 * j + q1].y;
        __syncthreads();
        z512i = lds[512];
    }
    // One pair at a time (its imaginary parts, |S| and split twiddle read one pair ahead).  The
    // partner bin's pre-split value goes to lane (64 - L) & 63, register 15 - m (16 - m on lane 0),
    // i.e. to the slot of Z[1024 - k]: a slot only this lane reads (512 is read by one instruction
    // of all lanes and rewritten by lane 0 only), so it is stored in place with no barrier; its
    // real part at once, its imaginary part after the next barrier.  INIT: X from the phases.
    double vmy[8];
    double zki = 0.0, zmi = 0.0;
    if constexpr (!INIT) {
        zki = lds[zb];
        zmi = lds[mb + 64 * 15];
        if (L == 0) zmi = zki;
    }
    // INIT: the phases U of the lane's bins (k, 1024 - k per pair, then 512), all issued up front
    double uk[8], um[8], u512 = 0.0;
    auto phase_of = [&](int k) -> double {
        return a.phase_u ? a.phase_u[((int64_t)b * NB + k) * a.Fmax + f]
                         : hash_uniform(a.seed, ((unsigned long long)b * NB + k) * 1048576ull + f);
    };
    // exp(2 pi i U) |S| with .real at DC and Nyquist (gl_iter_kernel's init_bin)
    auto phase_bin = [&](int k, double sv, double u) -> double2 {
        double sn, cs;
        sincospi(2.0 * u, &sn, &cs);
        return double2{sv * cs, (k == 0 || k == NB - 1) ? 0.0 : sv * sn};
    };
    if constexpr (INIT) {
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            uk[m] = phase_of(L + 64 * m);
            um[m] = phase_of(NH - L - 64 * m);
        }
        u512 = phase_of(512);
    }
    double sa = buf_f32(rS, 4 * L), sb = buf_f32(rS, 4 * (NH - L));
    // split twiddles t[k] = W2048^(L + 64 m) = W2048^L x W32^m (compile-time W32^m)
    const double2 tL = buf_c64(rT, 16 * L, 0);
    double2 tk = tL;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        __builtin_amdgcn_sched_barrier(0);
        const int k = L + 64 * m;
        double zki_n = 0.0, zmi_n = 0.0, sa_n, sb_n = 0.0;
        double2 tk_n = double2{0.0, 0.0};
        if (m < 7) {
            if constexpr (!INIT) {
                zki_n = lds[zb + 64 * (m + 1)];
                zmi_n = lds[mb + 64 * (14 - m)];
            }
            sa_n = buf_f32s(rS, 4 * L, 256 * (m + 1));
            sb_n = buf_f32(rS, 4 * (NH - k - 64));
            tk_n = cmulf(tL, double2{kW32[m + 1][0], kW32[m + 1][1]});
        } else {
            sa_n = buf_f32s(rS, 0, 2048);  // k = 512
            tk_n = buf_c64(rT, 0, 8192);  // k = 512
        }
        double2 xk, xm;
        if constexpr (INIT) {
            xk = phase_bin(k, sa, uk[m]);
            xm = phase_bin(NH - k, sb, um[m]);
        } else {
            // 2E = Z[k] + conj Z[N-k], 2O = -i (Z[k] - conj Z[N-k]): X[k] = E + t O up to the factor 2
            const double2 E = double2{zkr[m] + zmr[m], zki - zmi};
            const double2 O = double2{zki + zmi, zmr[m] - zkr[m]};
            const double2 tO = cmulf(O, tk);
            xk = unit_phase(cadd(E, tO), sa);         // X[k]
            xm = unit_phase(cconj(csub(E, tO)), sb);  // X[1024 - k]
        }
        if ((L | m) == 0) {  // istft: .real of the Hermitian extension at DC and Nyquist
            xk.y = 0.0;
            xm.y = 0.0;
        }
        // the pair's two pre-splits share E, D and O: the partner's (conj t' = -t of bin 1024 - k)
        // is (E.x + O.y, O.x - E.y), E = X[k] + conj X[N-k], O = (X[k] - conj X[N-k]) conj(t)
        const double2 Ep = double2{xk.x + xm.x, xk.y - xm.y};
        const double2 Op = cmulcf(double2{xk.x - xm.x, xk.y + xm.y}, tk);
        v[m] = double2{Ep.x - Op.y, Ep.y + Op.x};
        const double2 vm = double2{Ep.x + Op.y, Op.x - Ep.y};
        lds[mb + 64 * (15 - m)] = vm.x;
        vmy[m] = vm.y;
        zki = zki_n;
        zmi = zmi_n;
        sa = sa_n;
        sb = sb_n;
        tk = tk_n;
    }
    __builtin_amdgcn_sched_barrier(0);
    double2 v512;
    {  // k = 512 pairs with itself: 2E = (2 Re Z, 0), 2O = (2 Im Z, 0)
        const double2 x = INIT ? phase_bin(512, sa, u512)
                               : unit_phase(double2{2.0 * z512r + 2.0 * z512i * tk.x, 2.0 * z512i * tk.y}, sa);
        v512 = inv_presplit2(x, x, tk);
    }
    lds[512] = v512.x;  // the same value from every lane
    __syncthreads();
#pragma unroll
    for (int R = 8; R < 16; ++R) v[R].x = lds[zb + 64 * R];
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 8; ++m)
        lds[mb + 64 * (15 - m)] = vmy[m];
    lds[512] = v512.y;
    __syncthreads();
#pragma unroll
    for (int R = 8; R < 16; ++R) v[R].y = lds[zb + 64 * R];
    __syncthreads();
    // ---- inverse FFT; z'[n] -> real samples 2n, 2n + 1; window the support and store float64
    // (the frame's store range is its support: stores outside it are dropped by the range check)
    wave_fft1024<true>(v, lds, t2, rT, L);
    // (samples 2 (16 r3 + K2) + 128 (j + 4 q1): the window by the same recurrence; each sample pair
    // is one 8-byte store (float32 pair; a wave's 64 pairs are 128 consecutive samples) into the
    // frame slot [fb, fb + winp), pairs outside the slot dropped by its range; the slot's one or two
    // samples outside the support are never read)
    const auto rO = buf_rsrc(static_cast<frame_t*>(a.next) + ((int64_t)b * a.Fmax + f) * g.winp, (unsigned)g.winp * 4);
    __builtin_amdgcn_sched_barrier(0);
    const double2 s0 = buf_c64(rC, 16 * L, 2048), s1 = buf_c64(rC, 16 * L, 3072);
    double a0 = s0.x, a1 = s0.y, b0 = s1.x, b1 = s1.y;
#pragma unroll
    for (int q1 = 0; q1 < 4; ++q1)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int s = 2 * (256 * q1 + 64 * j + 16 * r3 + K2);
            const double2 z = v[4 * j + q1];
            // (1/2 of the pre-split) x 1/NH: one exact power-of-two scale
            const float2 o2 = float2{(float)(fma(-0.5, a0, 0.5) * (z.x * (0.5 / NH))),
                                     (float)(fma(-0.5, b0, 0.5) * (z.y * (0.5 / NH)))};
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o2), rO, (s - g.fb) * 4, 0, 0);
            const double a2 = fma(K, a1, -a0), b2 = fma(K, b1, -b0);
            a0 = a1;
            a1 = a2;
            b0 = b1;
            b1 = b2;
        }
}

// ---------------------------------------------------------------- persistent GL loop (small batches)
// Every GL iteration after the initial one, for all frames (<= 512 in all), in ONE launch: one
// workgroup per (sentence, frame) keeps its iteration-invariant operands (|S| row, window,
// twiddles, and the overlap-add geometry of its 2048 STFT input samples: contributor offsets and
// the window sum-square) in registers.  Frames are 8-byte granules {tag | float32 sample} (gran_t)
// in two ping-pong slots: iteration it reads slot it & 1 (tag it), writes slot (it + 1) & 1.
// Per iteration each thread re-reads the granules of its 8 input samples' <= 5 contributors until
// every tag is the iteration's (the neighbour wait and the overlap-add loads are one), then
// STFT -> S X/|X| -> iSTFT as gl_iter_kernel, and stores its frame's samples: no flag words, no
// per-frame publish.  Overwriting slot (it + 1) & 1 is safe because the contributor relation is
// symmetric (checked on the host for the geometry and frame count, gl_persistent_path): every
// reader of this frame's iteration it - 1 output is one of its own contributors, whose iteration
// it output this frame has read - so that reader has finished its iteration it - 1 gather.
// Placement: every workgroup publishes its XCD; frames map to XCDs in contiguous runs over the
// runtime placement.  A frame whose consumers (frames within 4; sentence edges excepted, where
// the STFT's reflection reaches further) share its XCD stores with workgroup scope (the line stays
// in that XCD's L2, where the consumers' sc1 loads read it); others write through (agent scope).
// A stale copy of a cross-XCD granule carries an old tag and is read again.  Waits are bounded.
struct PersArgs {
    IterArgs it;        // S, F, Fmax, B, geometry, constants (y / next / prev unused)
    gran_t* frames;     // [2][B][Fmax][winp]
    int64_t fstride;    // granules per slot
    int iters;          // iterations after the initial one
    unsigned* xtab;     // [B][Fmax] each workgroup's XCD, salted (zeroed by the initial iSTFT)
    unsigned salt;      // per launch (18 bits): tag(it) = salt << 14 | it
    long long tmo;      // wall_clock64 ticks per wait
    int* status;
    long long* prof;    // diagnostic (TTS_GL_PHASES): per-phase wall_clock64 ticks of frame prof_f, or null
    int prof_f;
    int nowait;         // measurement only (TTS_GL_NOWAIT=1): one gather sweep, tags unchecked (wrong results)
    int first_sleep;    // s_sleep(4) count before an iteration's first gather poll (TTS_GL_FIRST_SLEEP)
    int drop_f;         // fault injection (tests, TTS_GL_INJECT_DROP): sentence 0's frame drop_f stops
                        // after its first iteration without storing it (-1: none)
};
constexpr int GL_SC1_VOLATILE = (int)0x80000010u;  // buffer aux: sc1 (bit 4) | volatile (bit 31)
constexpr int GL_OOB_OFF = 0x7FFFFFF0;               // past every granule buffer: reads 0, no access
constexpr int GL_DMAX = 4;                            // overlap-add contributors lie within 4 frames
constexpr int GL_SLOTS = 2 * GL_DMAX + 1;              // gather buffer slots (frames f-4 .. f+4)
constexpr int GL_PAIRS = 9;                            // granule pairs per thread (<= 2304 per frame:
                                                       // 2216 at most for n_fft 2048 / win 1102 / hop 275)
// fill word of a fresh (or salt-wrapped) granule buffer, every dword: tag 1 = salt 0, never a live tag
constexpr unsigned GL_GRAN_FILL = 1u;
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) unsigned gu32_t;
typedef __attribute__((address_space(1))) int gi32_t;

// TWO: the form for 257..512 frames, two workgroups per compute unit (one wave per SIMD each):
// at most 256 registers per lane (the FFT twiddles read pass by pass, fft1024_regs_gtw, instead of
// 48 VGPRs for the whole loop) and the spectrum X in the FFT buffer the forward transform does not
// end in, so the static LDS halves.  Same values, same operations: bitwise the one-per-CU form.
template <bool TWO>
__device__ __forceinline__ void gl_persistent_body(const PersArgs& p) {
    const IterArgs& a = p.it;
    const int b = blockIdx.y;
    const int Fb = a.F[b];
    if ((int)blockIdx.x >= Fb) return;  // (a speculative batch-1 run sizes the grid as an upper bound)
    const Geo g = a.g;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ __align__(16) double2 buf0[NH];  // forward wave regions, then the spectrum X
    __shared__ __align__(16) double2 buf1[NH];  // Z, then the inverse wave regions
    __shared__ int sh[4];  // frame, local stores, abort
    auto fail = [&](int code) {
        __hip_atomic_store((gi32_t*)p.status, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sh[2] = 1;
    };
    if (tid == 0) sh[2] = 0;
    // ---- placement: frames -> XCDs in contiguous runs over where the workgroups actually run
    int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7;
    unsigned* xt = p.xtab + (int64_t)b * a.Fmax;
    if (tid == 0)
        __hip_atomic_store((gu32_t*)(xt + blockIdx.x), (p.salt << 8) | (unsigned)xcc, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    constexpr int PV = TWO ? 8 : 4;  // table entries per lane (Fb <= 64 PV)
    if (wave == 0) {
        unsigned v[PV];  // blocks PV lane .. PV lane + PV - 1
        long long t_end = 0;
        bool ok = true;
        for (int spin = 0;; ++spin) {
            ok = true;
#pragma unroll
            for (int i = 0; i < PV; ++i) {
                const int k = lane * PV + i;
                v[i] = k < Fb ? __hip_atomic_load((gu32_t*)(xt + k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
                ok = ok && (k >= Fb || (v[i] >> 8) == p.salt);
            }
            if (__all(ok)) break;
            if (spin == 0) {
                t_end = (long long)wall_clock64() + p.tmo;
            } else if ((spin & 31) == 0 && (long long)wall_clock64() > t_end) {
                break;
            }
        }
        int base = 0, cnt = 0, rank = 0;
        for (int x = 0; x < 8; ++x) {
            int c = 0, r = 0;
#pragma unroll
            for (int i = 0; i < PV; ++i) {
                const int k = lane * PV + i;
                const bool on = k < Fb && (int)(v[i] & 7) == x;
                c += __popcll(__ballot(on));
                r += __popcll(__ballot(on && k < (int)blockIdx.x));
            }
            if (x < xcc) base += c;
            if (x == xcc) { cnt = c; rank = r; }
        }
        if (lane == 0) {
            const int f = base + rank;
            sh[0] = f;
            sh[1] = f - 4 >= base && f + 4 < base + cnt && f >= 5 && f <= Fb - 6;
            if (!__all(ok)) fail(2);
        }
    }
    __syncthreads();
    if (sh[2]) return;
    const int f = sh[0];
    const bool local = sh[1];
    constexpr int PN = NFFT / GL_THREADS;
    // ---- iteration-invariant operands
    const spec_t* Sf = a.S + ((int64_t)b * a.Fmax + f) * NB;
    // the FFT twiddles in registers for the whole loop (one wave per SIMD: no occupancy to lose;
    // table reads where used cost latency on every pass here); TWO: read from the table
    std::conditional_t<TWO, TwMix, TwRegs> twf;
    twf.load(a.c.tw);  // (TWO: the table pointers are re-laundered every iteration: no hoisted pass reads)
    __shared__ __align__(16) double2 tw_pass[TWO ? TW_LDS : 1];
    if constexpr (TWO) TwMix::fill(tw_pass, a.c.tw);  // (ordered before its first use by the barriers below)
    // split twiddles (TWO: read from the table where used) and |S| of the thread's bins
    // k = bin2l(r) (layout B); thread 0 also holds the Nyquist bin's
    double2 tk[4];
    spec_t sk[4];  // (|S| in its float storage: widened where it is used)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        tk[r] = a.c.tw[bin2l(r)];
        sk[r] = Sf[bin2l(r)];
    }
    auto tkf = [&](int r) { return tk[r]; };
    const double2 tnyq = !TWO && tid == 0 ? a.c.tw[NH] : double2{0.0, 0.0};  // (TWO: from the table)
    const spec_t snyq = tid == 0 ? Sf[NH] : 0.f;
    // STFT input sample i of this thread: n = edge_sample(tid, i); its overlap-add contributors and
    // window sum-square, as ola_sample.  A contributor is an index into the gather buffer og: slot
    // s = fi - f + GL_DMAX holds frame fi's granule values (every contributor lies within GL_DMAX
    // frames, reflection included: checked here), index og_zero a 0.0 for absent ones.
    const int N = g.hop * (Fb - 1);
    extern __shared__ __align__(16) float og[];  // [GL_SLOTS][winp] + 2
    const int og_zero = GL_SLOTS * g.winp;
    __shared__ int rlo[GL_SLOTS], rhi[GL_SLOTS], rpre[GL_SLOTS + 1];
    if (tid < GL_SLOTS) {
        rlo[tid] = 0x7FFFFFFF;
        rhi[tid] = -1;
    }
    if (tid < 2) og[og_zero + tid] = 0.f;
    __syncthreads();
    double wi[PN];  // the window at this thread's samples: analysis (input) and synthesis (output) alike
    // contributor LDS indices, two 16-bit halves per register (og_zero < 65536: checked below)
    constexpr int OP = (OLA_MAX + 1) / 2;
    unsigned offp[PN][OP];
    float wssv[PN];
    if (og_zero > 0xFFFF) fail(6);
#pragma unroll
    for (int i = 0; i < PN; ++i) {
        const int n = edge_sample(tid, i);
        const bool sup = n >= g.woff && n < g.woff + g.win;
        wi[i] = sup ? a.c.win[n] : 0.0;
        const int q = reflect_idx(f * g.hop + n - NFFT / 2, N) + NFFT / 2;
        int ilo = q - g.woff - g.win + 1;
        ilo = ilo <= 0 ? 0 : (ilo + g.hop - 1) / g.hop;
        int ihi = (q - g.woff) / g.hop;
        if (ihi > Fb - 1) ihi = Fb - 1;
        const bool any = sup && q >= g.woff;
        float wss = 0.f;
#pragma unroll
        for (int k = 0; k < OP; ++k) offp[i][k] = 0u;
#pragma unroll
        for (int k = 0; k < OLA_MAX; ++k) {
            const int fi = ilo + k;
            const int o = q - fi * g.hop;
            const bool ok = any && fi <= ihi;
            const int sl = fi - f + GL_DMAX, gg = o - g.fb;
            if (ok && (sl < 0 || sl >= GL_SLOTS)) fail(4);  // (never: contributors are within GL_DMAX)
            const bool in = ok && sl >= 0 && sl < GL_SLOTS;
            offp[i][k >> 1] |= (unsigned)(in ? sl * g.winp + gg : og_zero) << (16 * (k & 1));
            if (in) {
                atomicMin(&rlo[sl], gg);
                atomicMax(&rhi[sl], gg);
            }
            wss = (float)((double)wss + (ok ? a.c.win2[o] : 0.0));
        }
        // (a sample whose sum-square is below FLT_MIN keeps its sum undivided: y / 1.0f == y)
        wssv[i] = wss > 1.17549435e-38f ? wss : 1.0f;
    }
    // The gather's loads: slot s needs granules [rlo, rhi] of frame f + s - GL_DMAX, read as
    // 16-byte-aligned pairs (winp is a multiple of 4: granule pairs start at even indices); pair u of
    // the workgroup goes to thread u % 256 (at most GL_PAIRS per thread).  gdst: LDS index | need
    // bits (bit 30: the pair's first granule is needed, bit 31: its second); pairs past the list
    // read out of range (zeros, to the zero word).
    __syncthreads();
    if (tid == 0) {
        int acc = 0;
        for (int sl = 0; sl < GL_SLOTS; ++sl) {
            rpre[sl] = acc;
            acc += rhi[sl] >= 0 ? (rhi[sl] - (rlo[sl] & ~1)) / 2 + 1 : 0;
        }
        rpre[GL_SLOTS] = acc;
        if (acc > GL_PAIRS * GL_THREADS) fail(5);
    }
    __syncthreads();
    // (a listed pair needs at least one of its granules; its source offset is the LDS index
    // rebased to frame f - GL_DMAX: slot sl of the gather buffer mirrors frame f + sl - GL_DMAX)
    unsigned gdst[GL_PAIRS];
#pragma unroll
    for (int m = 0; m < GL_PAIRS; ++m) {
        const int u = tid + m * GL_THREADS;
        gdst[m] = (unsigned)og_zero;
        if (u < rpre[GL_SLOTS]) {
            int sl = 0;
            while (u >= rpre[sl + 1]) ++sl;
            const int g0 = (rlo[sl] & ~1) + 2 * (u - rpre[sl]);
            gdst[m] = (unsigned)(sl * g.winp + g0) | (g0 >= rlo[sl] ? 1u << 30 : 0u) | (g0 + 1 <= rhi[sl] ? 1u << 31 : 0u);
        }
    }
    const int gbase = (f - GL_DMAX) * g.winp * 8;
    auto goff = [&](int m) {
        return (gdst[m] >> 30) ? gbase + (int)(gdst[m] & 0x3FFFFFFFu) * 8 : GL_OOB_OFF;
    };
    // byte offset of output sample i's granule in the frame slot (computed where stored); samples
    // outside the window support take an out-of-range offset (the buffer store drops them)
    // (TWO: computed where stored, from an opaque thread index: held, they would not fit)
    auto soff_of = [&](int t, int i) {
        const int e = edge_sample(t, i);
        return (unsigned)(e - g.woff) < (unsigned)g.win ? (e - g.fb) * 8 : GL_OOB_OFF;
    };
    int soffv[TWO ? 1 : PN];
    if constexpr (!TWO) {
#pragma unroll
        for (int i = 0; i < PN; ++i) soffv[i] = soff_of(tid, i);
    }
    auto soff = [&](int i) { if constexpr (TWO) return soff_of(tid_opaque(), i); else return soffv[i]; };
    const bool timed = p.prof && f == p.prof_f && b == 0 && tid == 0;
    long long ph[6] = {0, 0, 0, 0, 0, 0};
    long long tp = timed ? (long long)wall_clock64() : 0;
#define GL_PHASE(k)                                      \
    if (timed) {                                         \
        const long long tn = (long long)wall_clock64(); \
        ph[k] += tn - tp;                                \
        tp = tn;                                         \
    }
    const unsigned tag0 = p.salt << 14;
    for (int it = 0; it < p.iters; ++it) {
        const gran_t* src = p.frames + (it & 1) * p.fstride + (int64_t)b * a.Fmax * g.winp;
        gran_t* dst = p.frames + ((it + 1) & 1) * p.fstride + ((int64_t)b * a.Fmax + f) * g.winp;
        const unsigned want = tag0 | (unsigned)it;
        if constexpr (TWO) {  // an opaque copy of the table pointer per iteration: loop-invariant table
            int z = 0;  // an opaque zero offset (the pointers keep their address spaces): table
            asm volatile("" : "+v"(z));  // reads hoisted out of the loop would not fit the registers
            twf.tw = (g_d*)a.c.tw + z;
            twf.pt = (l_d*)tw_pass + z;
        }
        // ---- gather: the workgroup's granule pairs (each thread <= GL_PAIRS 16-byte sc1 loads, all in
        // flight at once), re-read until every needed tag is this iteration's, then into LDS
        {
            const auto rG = buf_rsrc(src, (unsigned)(a.Fmax * g.winp * 8));
            long long t_end = 0;
            u32x4 x[GL_PAIRS];
            // (a poll storm from every workgroup the moment it has stored slows the stores it waits for)
            for (int i = 0; i < p.first_sleep; ++i) __builtin_amdgcn_s_sleep(4);
            for (int spin = 0;; ++spin) {
#pragma unroll
                for (int m = 0; m < GL_PAIRS; ++m)
                    x[m] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rG, goff(m), 0, GL_SC1_VOLATILE));
                bool ok = true;
#pragma unroll
                for (int m = 0; m < GL_PAIRS; ++m)
                    ok = ok && (!(gdst[m] & (1u << 30)) || x[m].y == want) && (!(gdst[m] & (1u << 31)) || x[m].w == want);
                if (__all(ok) || p.nowait) break;
                if (spin == 0) {
                    t_end = (long long)wall_clock64() + p.tmo;
                } else if ((spin & 31) == 0 && (long long)wall_clock64() > t_end) {
                    if (lane == 0) fail(1);
                    break;
                }
                if (GLP_SLEEP) __builtin_amdgcn_s_sleep(GLP_SLEEP);
            }
            // (unneeded granules of a pair land on LDS words no sum reads; out-of-range pairs write
            // zeros to the zero word)
#pragma unroll
            for (int m = 0; m < GL_PAIRS; ++m)
                *reinterpret_cast<float2*>(og + (gdst[m] & 0x3FFFFFFFu)) =
                    float2{__uint_as_float(x[m].x), __uint_as_float(x[m].z)};
        }
        __syncthreads();  // the gather buffer (or a timeout) before the sums and the FFT's LDS passes
        if (sh[2]) return;
        GL_PHASE(0)
        // ---- overlap-add sums (librosa istft: float64 contributions into a float32 signal, frame
        // order) straight into the forward FFT's layout-A registers
        double2 v[4];
#pragma unroll
        for (int i = 0; i < PN; ++i) {
            // (absent contributors read the zero word: adding +0.0 leaves the sum bitwise unchanged,
            // which is never -0.0)
            float y = 0.f;
#pragma unroll
            for (int k = 0; k < OLA_MAX; ++k) y = (float)((double)y + (double)og[(offp[i][k >> 1] >> (16 * (k & 1))) & 0xFFFFu]);
            const float yv = y / wssv[i];
            if (i & 1) v[i >> 1].y = wi[i] * (double)yv;
            else v[i >> 1].x = wi[i] * (double)yv;
        }
        GL_PHASE(1)
        fft2l_fwd(v, buf0, twf);
        GL_PHASE(2)
        double2 xnyq = double2{0.0, 0.0};
        spectrum2l(v, buf1, tkf, [&](int r) { return (double)sk[r]; }, TWO ? twf.tw_at(NH) : tnyq, (double)snyq, xnyq);
        presplit2l(v, buf0, tkf, xnyq);
        GL_PHASE(3)
        fft2l_inv(v, buf1, twf);
        GL_PHASE(4)
        if (b == 0 && f == p.drop_f) return;  // fault injection only: never stores iteration 1
        // ---- the frame's samples, tagged with the next iteration: XCD-local (workgroup-scope store,
        // the line stays in the XCD's L2) when every consumer shares this XCD, else written through
        const unsigned nt = tag0 | (unsigned)(it + 1);
        const auto rD = buf_rsrc(dst, (unsigned)g.winp * 8);
        // one 16-byte store per sample pair (2n, 2n + 1): two whole granules; a pair straddling an
        // end of the support also writes the slot's sample outside it (never read)
#pragma unroll
        for (int r = 0; r < PN / 2; ++r) {
            const u32x4 gv = u32x4{__float_as_uint((float)(wi[2 * r] * (v[r].x * (1.0 / NH)))), nt,
                                   __float_as_uint((float)(wi[2 * r + 1] * (v[r].y * (1.0 / NH)))), nt};
            const int e = edge_sample(TWO ? tid_opaque() : tid, 2 * r);
            const int off = e + 1 >= g.woff && e < g.woff + g.win ? (e - g.fb) * 8 : GL_OOB_OFF;
            // plain (workgroup-scope) store: the line stays in this XCD's L2; sc1: written through
            if (local) __builtin_amdgcn_raw_buffer_store_b128(gv, rD, off, 0, 0);
            else __builtin_amdgcn_raw_buffer_store_b128(gv, rD, off, 0, 0x10);
        }
        GL_PHASE(5)
    }
#undef GL_PHASE
    if (timed)
        for (int k = 0; k < 6; ++k) p.prof[k] = ph[k];
}
__global__ __launch_bounds__(GL_THREADS) void gl_persistent_kernel(const PersArgs p) { gl_persistent_body<false>(p); }
__global__ __launch_bounds__(GL_THREADS) __attribute__((amdgpu_waves_per_eu(2, 2))) void gl_persistent2_kernel(
    const PersArgs p) {
    gl_persistent_body<true>(p);
}

// the initial iSTFT's granules (slot 0) as float32 frames for the fused loop, when the persistent
// launch could not be placed
__global__ void gl_gran_to_frames_kernel(const gran_t* in, float* out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = __uint_as_float((unsigned)in[i].v);
}

// ---------------------------------------------------------------- final OLA + inverse pre-emphasis
struct FinArgs {
    const void* frames;  // frame_t (fused / batched loops) or gran_t (persistent): gl_ola_kernel<FT>
    const int* F;
    int Fmax, B;
    Geo g;
    GLConst c;
    float* y;  // [B][Nmax]
    int64_t Nmax;
    const int* status;  // the persistent loop's status word, or null: nonzero poisons the signal (NaN)
    int* host_status;   // pinned host word the status is copied to by thread 0 of block (0, 0), or null
    int* host_seq;      // ... then (pipeline mode) this pinned word is set to `seq` (release), or null
    int seq;
    const float* wssp;  // [hop] float32 window sum-square of a sample whose every contributing frame
                        // exists, by (q - woff) mod hop (summed on the host in ola_sample's order)
};

template <typename FT>
__global__ void gl_ola_kernel(const FinArgs a) {
    const int b = blockIdx.y;
    const int Fb = a.F[b];
    const int N = a.g.hop * (Fb - 1);
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (a.host_status && p == 0 && b == 0) {  // the persistent loop's status, for the host's collect
        __hip_atomic_store(a.host_status, *a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (a.host_seq) release_word_system(a.host_seq, a.seq);
    }
    if (p >= N) return;
    // a persistent loop whose hand-off wait timed out left frames unwritten: never hand out a
    // plausible-looking waveform for it (the run's error status is raised when it is collected)
    const bool bad = a.status && *a.status != 0;
    // (contributor loads issued together when the geometry allows it: bitwise the same sum; the
    // window sum-square from the periodic table where no contributor is clipped, as ola_sample
    // would sum it, else summed here)
    const FT* fr = static_cast<const FT*>(a.frames) + (int64_t)b * a.Fmax * a.g.winp;
    const Geo& g = a.g;
    const int q = p + NFFT / 2;
    float yv;
    if ((g.win + g.hop - 1) / g.hop <= OLA_MAX && q >= g.woff) {
        const int u = q - g.woff;
        const int ihu = u / g.hop;
        int ilo = u - g.win + 1;
        const bool full = ilo >= 1 && ihu <= Fb - 1;
        ilo = ilo <= 0 ? 0 : (ilo + g.hop - 1) / g.hop;
        const int ihi = ihu > Fb - 1 ? Fb - 1 : ihu;
        double fv[OLA_MAX];
#pragma unroll
        for (int k = 0; k < OLA_MAX; ++k) {
            const int i = ilo + k;
            fv[k] = i <= ihi ? fval(fr[(int64_t)i * g.winp + (q - i * g.hop - g.fb)]) : 0.0;
        }
        float y = 0.f, wss = 0.f;
#pragma unroll
        for (int k = 0; k < OLA_MAX; ++k) y = (float)((double)y + fv[k]);
        if (full) {
            wss = a.wssp[u - ihu * g.hop];
        } else {
            for (int i = ilo; i <= ihi; ++i) wss = (float)((double)wss + a.c.win2[q - i * g.hop]);
        }
        yv = wss > 1.17549435e-38f ? y / wss : y;
    } else {
        yv = ola_sample(fr, q, Fb, g, a.c.win2);
    }
    a.y[(int64_t)b * a.Nmax + p] = bad ? __builtin_nanf("") : yv;
}

// gl_ola_kernel<frame_t> with OLA_R samples per thread (stride 256) and every contributor load
// (and window sum-square load) of the thread issued before the first sum: at one sample per
// thread a wave held ~1.3 KB of loads in flight, and the launch ran at ~2.9 TB/s (latency-bound by
// bytes in flight; configs[4]: 442 MB per launch).  Per sample the same loads and the same
// double-rounded sum order as gl_ola_kernel: bitwise equal.  Needs the unrolled geometry
// (ola_multi_ok).
constexpr int OLA_R = 4;
__device__ __forceinline__ int div_small(int n, int d, float rd) {  // floor(n / d), 0 <= n < 2^24
    int qt = (int)((float)n * rd);
    const int r = n - qt * d;
    qt += r >= d ? 1 : 0;
    qt -= r < 0 ? 1 : 0;
    return qt;
}
__global__ __launch_bounds__(256) void gl_ola_multi_kernel(const FinArgs a) {
    const int b = blockIdx.y;
    const int Fb = a.F[b];
    const Geo& g = a.g;
    const int N = g.hop * (Fb - 1);
    const int p0 = blockIdx.x * (256 * OLA_R) + threadIdx.x;
    if (a.host_status && p0 == 0 && b == 0) {
        __hip_atomic_store(a.host_status, *a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (a.host_seq) release_word_system(a.host_seq, a.seq);
    }
    if (p0 >= N) return;
    const bool bad = a.status && *a.status != 0;
    const float* fr = static_cast<const float*>(a.frames) + (int64_t)b * a.Fmax * g.winp;
    const float rhop = __builtin_amdgcn_rcpf((float)g.hop);
    const int step = g.winp - g.hop;  // frame i's element for sample q: i (winp - hop) + q - fb
    float fv[OLA_R][OLA_MAX], wv[OLA_R];
    int ilo[OLA_R], ihi[OLA_R];
#pragma unroll
    for (int j = 0; j < OLA_R; ++j) {
        const int q = p0 + 256 * j + NFFT / 2, u = q - g.woff;
        const int ihu = div_small(u, g.hop, rhop);
        int lo = u - g.win + 1;
        const bool full = lo >= 1 && ihu <= Fb - 1;
        lo = lo <= 0 ? 0 : div_small(lo + g.hop - 1, g.hop, rhop);
        const int hi = p0 + 256 * j < N ? min(ihu, Fb - 1) : -1;
        ilo[j] = lo;
        ihi[j] = hi;
        const int o = lo * step + q - g.fb;
#pragma unroll
        for (int k = 0; k < OLA_MAX; ++k) fv[j][k] = lo + k <= hi ? fr[o + k * step] : 0.f;
        wv[j] = full && hi >= 0 ? a.wssp[u - ihu * g.hop] : -1.f;  // -1: sum the window here
    }
#pragma unroll
    for (int j = 0; j < OLA_R; ++j) {
        const int p = p0 + 256 * j;
        if (p >= N) break;
        const int q = p + NFFT / 2;
        float y = 0.f;
#pragma unroll
        for (int k = 0; k < OLA_MAX; ++k) y = (float)((double)y + (double)fv[j][k]);
        float wss = wv[j];
        if (wss < 0.f) {
            wss = 0.f;
            for (int i = ilo[j]; i <= ihi[j]; ++i) wss = (float)((double)wss + a.c.win2[q - i * g.hop]);
        }
        const float yv = wss > 1.17549435e-38f ? y / wss : y;
        a.y[(int64_t)b * a.Nmax + p] = bad ? __builtin_nanf("") : yv;
    }
}
bool ola_multi_ok(const Geo& g, int64_t Nmax) {
    return (g.win + g.hop - 1) / g.hop <= OLA_MAX && g.woff <= NFFT / 2 && Nmax + NFFT < (1 << 24) &&
           (Nmax / g.hop + 2) * (int64_t)g.winp < (1ll << 31);  // (int frame offsets)
}
// the overlap-add of float32 frames (the fused / batched loops' slots) into the signal
void launch_ola_frames(const FinArgs& f, hipStream_t s) {
    static const bool single = [] {  // measurement: TTS_GL_OLA_SINGLE=1, one sample per thread
        const char* v = getenv("TTS_GL_OLA_SINGLE");
        return v && v[0] == '1';
    }();
    if (!single && ola_multi_ok(f.g, f.Nmax))
        hipLaunchKernelGGL(gl_ola_multi_kernel, dim3((unsigned)((f.Nmax + 256 * OLA_R - 1) / (256 * OLA_R)), f.B),
                           dim3(256), 0, s, f);
    else
        hipLaunchKernelGGL(gl_ola_kernel<frame_t>, dim3((unsigned)((f.Nmax + 255) / 256), f.B), dim3(256), 0, s, f);
}

// y[n] = x[n] + c*y[n-1] in float64 (scipy.signal.lfilter([1], [1, -c], x), utils/audio.py:133-136).
// Chunk-parallel: workgroup (chunk i, sentence b) writes y[i*chunk, (i+1)*chunk) and starts its scan
// `look` samples earlier from y = 0: the state it misses is c^look * y, below 1e-22 of |y| (the host
// picks look from |c|; with look = 0 the one workgroup per sentence scans from sample 0, exactly the
// recurrence up to rounding order).  A tile of SCAN_THREADS*SCAN_PER samples: per-thread serial scan,
// then the (c^len, value) carries composed across lanes by shuffles and across waves through LDS.
__device__ __forceinline__ void scan_combine(double& A, double& Bv, double pa, double pb) {
    // (pa, pb) precedes (A, Bv): y_out = A (pa y_in + pb) + Bv
    Bv = fma(pb, A, Bv);
    A = pa * A;
}
__global__ __launch_bounds__(SCAN_THREADS) void preemph_scan_kernel(const float* y, int64_t Nmax, const int* F, int hop,
                                                                    double coef, int apply, int64_t chunk, int64_t look,
                                                                    double* wav) {
    const int b = blockIdx.y;
    const int64_t N = (int64_t)hop * (F[b] - 1);
    const int64_t o0 = (int64_t)blockIdx.x * chunk;
    if (o0 >= N) return;
    const int64_t o1 = o0 + chunk < N ? o0 + chunk : N;
    const float* x = y + (int64_t)b * Nmax;
    double* o = wav + (int64_t)b * Nmax;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (!apply) {
        for (int64_t i = o0 + tid; i < o1; i += SCAN_THREADS) o[i] = (double)x[i];
        return;
    }
    constexpr int TILE = SCAN_THREADS * SCAN_PER, NW = SCAN_THREADS / 64;
    __shared__ double wa[NW], wb[NW];
    double cpow[SCAN_PER + 1];
    cpow[0] = 1.0;
#pragma unroll
    for (int k = 1; k <= SCAN_PER; ++k) cpow[k] = cpow[k - 1] * coef;
    const int64_t s0 = o0 - look > 0 ? ((o0 - look) & ~(int64_t)7) : 0;
    double carry = 0.0;  // y at the end of the previous tile
    for (int64_t t0 = s0; t0 < o1; t0 += TILE) {
        const int64_t base = t0 + (int64_t)tid * SCAN_PER;
        double v = 0.0, loc[SCAN_PER];
#pragma unroll
        for (int k = 0; k < SCAN_PER; ++k) {
            v = (base + k < o1 ? (double)x[base + k] : 0.0) + coef * v;
            loc[k] = v;
        }
        // inclusive composition over the lanes of this wave
        double A = cpow[SCAN_PER], Bv = v;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const double pa = __shfl_up(A, off, 64), pb = __shfl_up(Bv, off, 64);
            if (lane >= off) scan_combine(A, Bv, pa, pb);
        }
        if (lane == 63) { wa[wave] = A; wb[wave] = Bv; }
        __syncthreads();
        // every wave composes the waves' totals itself (NW lanes), then takes its carry-in
        double WA = lane < NW ? wa[lane] : 1.0, WB = lane < NW ? wb[lane] : 0.0;
#pragma unroll
        for (int off = 1; off < NW; off <<= 1) {
            const double qa = __shfl_up(WA, off, 64), qb = __shfl_up(WB, off, 64);
            if (lane >= off) scan_combine(WA, WB, qa, qb);
        }
        const double win_in = wave == 0 ? carry : __shfl(WA, wave - 1, 64) * carry + __shfl(WB, wave - 1, 64);
        const double tile_end = __shfl(WA, NW - 1, 64) * carry + __shfl(WB, NW - 1, 64);
        // y entering this thread: compose the lanes before it (exclusive) with the wave's carry-in
        const double pa = __shfl_up(A, 1, 64), pb = __shfl_up(Bv, 1, 64);
        const double cin = lane == 0 ? win_in : pa * win_in + pb;
#pragma unroll
        for (int k = 0; k < SCAN_PER; ++k) {
            const int64_t i = base + k;
            if (i >= o0 && i < o1) o[i] = loc[k] + cpow[k + 1] * cin;
        }
        carry = tile_end;
        __syncthreads();  // wa / wb are rewritten by the next tile
    }
}

// ---------------------------------------------------------------- mel analysis
// AudioProcessor.melspectrogram (utils/audio.py:146-152) for the GST style wav
// (utils/synthesis.py:28-35): pre-emphasis FIR (lfilter([1, -c], [1]), :128-131) -> librosa 0.6.2
// stft (centre reflect pad, periodic Hann, float64 FFT, complex64 result) -> |D| (float32) ->
// mel_basis . |D| (float64) -> 20 log10(max(min_level, .)) - ref_level_db -> _normalize (:79-94).
// One workgroup per (sentence, frame); output frame-major [B][Fmax][num_mels] float32.
struct MelArgs {
    const double* wav;  // [B][Nmax]
    int64_t Nmax;
    const int* N;       // [B] samples
    int Fmax;
    Geo g;
    GLConst c;
    const double* basis;  // [num_mels][1025]
    int n_mels;
    double coef;          // pre-emphasis (0: none)
    double min_level, min_db, ref_db, max_norm;
    int signal_norm, symmetric, clip;
    float* mel;           // [B][Fmax][n_mels]
};

__global__ __launch_bounds__(GL_THREADS) void mel_analysis_kernel(const MelArgs a) {
    const int b = blockIdx.y, f = blockIdx.x;
    const int N = a.N[b];
    const int F = 1 + N / a.g.hop;
    if (f >= F) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ __align__(16) double2 buf0[NH];
    __shared__ __align__(16) double2 buf1[NH];
    __shared__ float mag[NB + 3];
    const FftTw ftw = load_fft_tw(a.c.tw);
    const double* y = a.wav + (int64_t)b * a.Nmax;
    constexpr int PN = NFFT / GL_THREADS;
    double* xr = reinterpret_cast<double*>(buf0);
#pragma unroll
    for (int i = 0; i < PN; ++i) {
        const int n = tid + i * GL_THREADS;
        // np.pad(y_pre, n_fft // 2, mode='reflect') of the pre-emphasised signal
        const int p = reflect_idx(f * a.g.hop + n - NFFT / 2, N);
        double v = y[p];
        if (a.coef != 0.0 && p > 0) v = v - a.coef * y[p - 1];
        xr[n] = a.c.win[n] * v;
    }
    __syncthreads();
    const double2* Z = fft1024<false>(buf0, buf1, ftw);
    for (int k = tid; k < NB; k += GL_THREADS) {
        const double2 zk = Z[k & (NH - 1)];
        const double2 zc = cconj(Z[(NH - k) & (NH - 1)]);
        const double2 E = double2{0.5 * (zk.x + zc.x), 0.5 * (zk.y + zc.y)};
        const double2 O = double2{0.5 * (zk.y - zc.y), -0.5 * (zk.x - zc.x)};
        const double2 t = a.c.tw[k];
        const float re = (float)(E.x + (t.x * O.x - t.y * O.y));  // stft result is complex64
        const float im = (float)(E.y + (t.x * O.y + t.y * O.x));
        mag[k] = hypotf(re, im);  // np.abs on complex64
    }
    __syncthreads();
    // mel bands: each wave owns bands wave, wave+4, ...; lanes stride the 1025 bins, float64
    for (int m = wave; m < a.n_mels; m += GL_THREADS / 64) {
        const double* row = a.basis + (int64_t)m * NB;
        double acc = 0.0;
        for (int k = lane; k < NB; k += 64) acc += row[k] * (double)mag[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
        if (lane == 0) {
            double S = 20.0 * log10(fmax(a.min_level, acc)) - a.ref_db;
            if (a.signal_norm) {
                S = (S - a.min_db) / -a.min_db;
                if (a.symmetric) {
                    S = (2.0 * a.max_norm) * S - a.max_norm;
                    if (a.clip) S = fmin(fmax(S, -a.max_norm), a.max_norm);
                } else {
                    S = a.max_norm * S;
                    if (a.clip) S = fmin(fmax(S, 0.0), a.max_norm);
                }
            }
            a.mel[((int64_t)b * a.Fmax + f) * a.n_mels + m] = (float)S;
        }
    }
}

bool getenv_off(const char* name) {
    const char* v = getenv(name);
    return v && v[0] == '0';
}

struct GraphKey {
    int B, Fmax, iters;
    bool operator<(const GraphKey& o) const { return std::tie(B, Fmax, iters) < std::tie(o.B, o.Fmax, o.iters); }
};

}  // namespace

struct tts_gl {
    tts_audio_config cfg{};
    Geo g{};
    hipStream_t stream = nullptr;
    hipEvent_t ev_in = nullptr, ev_out = nullptr, ev_t0 = nullptr, ev_t1 = nullptr;
    hipEvent_t ev_done = nullptr;  // end of the last tts_gl_run (its status copy included)
    double *win = nullptr, *win2 = nullptr, *pinv = nullptr, *basis = nullptr;
    int* NS = nullptr;  // mel analysis: samples per sentence
    int NS_cap = 0;
    double2* tw = nullptr;
    double2* wt = nullptr;  // gl_iter_wave_kernel pass-2 twiddles [16][4]
    double2* winc = nullptr;  // gl_iter_wave_kernel window rotation bases [4][64]
    float* wssp = nullptr;    // gl_ola_kernel periodic window sum-square [hop]
    double wrot = 0.0;
    bool wave = true;       // batched iterations on gl_iter_wave_kernel (TTS_GL_WAVE=0: gl_iter_kernel)
    // workspace
    size_t S_n = 0, fr_n = 0, y_n = 0;
    spec_t* S = nullptr;
    void* frames = nullptr;  // frame_t ping-pong slots
    float* y = nullptr;
    int* F = nullptr;
    int Fcap_B = 0;
    std::map<GraphKey, hipGraphExec_t> graphs;
    float last_ms = 0.f;
    int last_launches = 0;
    bool last_fused = false;
    bool last_persistent = false;
    int last_path = TTS_GL_PATH_UNFUSED;
    unsigned* flags = nullptr;  // persistent loop: [flags_n] the workgroups' XCD table
    size_t flags_n = 0;
    gran_t* pgr = nullptr;      // persistent loop: two granule slots
    size_t pgr_n = 0;
    std::vector<signed char> gather_fit;  // by frame count: the persistent gather's layout holds (-1: unknown)
    int* pstatus = nullptr;     // [dev] status of the persistent loop
    int* host_status = nullptr; // pinned coherent: [0] status of the last persistent loop, [1] its sequence
    int seq = 0;                // pipeline mode: the sequence the last persistent run's overlap-add sets
    hipStream_t seq_stream = nullptr;
    unsigned salt = 0;
    long long tmo = 0;
    bool have_last = false;
    IterArgs last_iter{};
    bool pipeline = false;        // tts_synth_run: caller's stream, completion collected later
    bool pending = false;         // a pipeline run whose timing / status is not collected yet
    bool last_timed = true;       // the last run recorded its events (not in pipeline mode)
    FinArgs last_fin{};
    size_t last_fstride = 0;
    // numpy-stream initial phases (tts_gl_set_phase_state, phase_mt.hip): the MT19937 state on the
    // device, the phases it drew for the current run, the stream and event of its last draw
    bool mt_armed = false;
    unsigned* mt_state = nullptr;  // [625] key + position
    double* mt_phase = nullptr;    // [B][1025][Fmax]
    size_t mt_phase_n = 0;
    int* mt_F = nullptr;           // tts_gl_draw_phases: the frame counts on the device
    int mt_F_n = 0;
    hipStream_t mt_stream = nullptr;
    hipEvent_t ev_mt = nullptr;
    MtWork mt_work;                // the draws' device workspace (phase_mt.hip)
    // tts_gl_save_pcm16: the peak word and the output offsets ([dev], host copy kept for the upload)
    unsigned long long* pcm_peak = nullptr;
    int64_t* pcm_start = nullptr;
    int pcm_start_n = 0;
    std::vector<int64_t> pcm_start_h;
};

extern "C" {

void tts_gl_destroy(tts_gl* g) {
    if (!g) return;
    if (g->stream) (void)hipStreamSynchronize(g->stream);
    if (g->ev_done) (void)hipEventSynchronize(g->ev_done);  // a pipeline run on another stream
    if (g->mt_stream) (void)hipEventSynchronize(g->ev_mt);  // the last numpy-stream phase draw
    mt_work_free(&g->mt_work);
    for (auto& kv : g->graphs) (void)hipGraphExecDestroy(kv.second);
    for (void* p : {(void*)g->win, (void*)g->win2, (void*)g->pinv, (void*)g->tw, (void*)g->S, (void*)g->frames,
                    (void*)g->y, (void*)g->F, (void*)g->basis, (void*)g->NS, (void*)g->flags, (void*)g->pstatus, (void*)g->pgr, (void*)g->wt, (void*)g->winc,
                    (void*)g->wssp, (void*)g->mt_state, (void*)g->mt_phase, (void*)g->mt_F, (void*)g->pcm_peak,
                    (void*)g->pcm_start})
        if (p) (void)hipFree(p);
    if (g->host_status) (void)hipHostFree(g->host_status);
    for (hipEvent_t e : {g->ev_in, g->ev_out, g->ev_t0, g->ev_t1, g->ev_done, g->ev_mt})
        if (e) (void)hipEventDestroy(e);
    if (g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
}

tts_status tts_gl_create(const tts_audio_config* cfg, const double* inv_mel_basis, void* stream, tts_gl** out) {
    TTS_CHECK(cfg && out, TTS_ERR_INVALID, "null argument");
    TTS_CHECK(cfg->n_fft == NFFT, TTS_ERR_UNSUPPORTED, "n_fft must be 2048 (num_freq 1025)");
    TTS_CHECK(cfg->win_length >= 2 && cfg->win_length <= NFFT, TTS_ERR_INVALID, "win_length must be in [2, n_fft]");
    TTS_CHECK(cfg->hop_length >= 1 && cfg->hop_length <= cfg->win_length, TTS_ERR_UNSUPPORTED,
              "hop_length must be in [1, win_length]");
    TTS_CHECK(cfg->num_mels >= 1 && cfg->num_mels <= 80, TTS_ERR_UNSUPPORTED, "num_mels must be <= 80");
    auto* g = new tts_gl();
    g->cfg = *cfg;
    g->g.hop = cfg->hop_length;
    g->g.win = cfg->win_length;
    g->g.woff = (NFFT - cfg->win_length) / 2;  // librosa util.pad_center
    g->g.fb = g->g.woff & ~1;
    g->g.winp = (cfg->win_length + (g->g.woff - g->g.fb) + 3) / 4 * 4;
    (void)stream;
    std::vector<double> win(NFFT, 0.0), win2(NFFT, 0.0);
    for (int n = 0; n < cfg->win_length; ++n) {
        const double w = 0.5 - 0.5 * std::cos(2.0 * M_PI * n / cfg->win_length);  // periodic Hann
        win[g->g.woff + n] = w;
        win2[g->g.woff + n] = w * w;
    }
    std::vector<double2> tw(NFFT);
    for (int m = 0; m < NFFT; ++m) tw[m] = double2{std::cos(2.0 * M_PI * m / NFFT), -std::sin(2.0 * M_PI * m / NFFT)};
    auto fail = [&](hipError_t e, const char* what) {
        tts_status st = hip_fail(e, what, __FILE__, __LINE__);
        tts_gl_destroy(g);
        return st;
    };
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking)) != hipSuccess) return fail(e, "stream");
    if ((e = hipEventCreateWithFlags(&g->ev_in, hipEventDisableTiming)) != hipSuccess) return fail(e, "event");
    if ((e = hipEventCreateWithFlags(&g->ev_out, hipEventDisableTiming)) != hipSuccess) return fail(e, "event");
    if ((e = hipEventCreateWithFlags(&g->ev_done, hipEventDisableTiming)) != hipSuccess) return fail(e, "event");
    if ((e = hipEventCreateWithFlags(&g->ev_mt, hipEventDisableTiming)) != hipSuccess) return fail(e, "event");
    if ((e = hipEventCreateWithFlags(&g->ev_t0, hipEventReleaseToDevice)) != hipSuccess) return fail(e, "event");
    if ((e = hipEventCreateWithFlags(&g->ev_t1, hipEventReleaseToDevice)) != hipSuccess) return fail(e, "event");
    if ((e = hipMalloc(&g->win, NFFT * 8)) != hipSuccess) return fail(e, "hipMalloc");
    if ((e = hipMalloc(&g->win2, NFFT * 8)) != hipSuccess) return fail(e, "hipMalloc");
    if ((e = hipMalloc(&g->tw, NFFT * sizeof(double2))) != hipSuccess) return fail(e, "hipMalloc");
    if ((e = hipMemcpy(g->win, win.data(), NFFT * 8, hipMemcpyHostToDevice)) != hipSuccess) return fail(e, "copy");
    if ((e = hipMemcpy(g->win2, win2.data(), NFFT * 8, hipMemcpyHostToDevice)) != hipSuccess) return fail(e, "copy");
    if ((e = hipMemcpy(g->tw, tw.data(), NFFT * sizeof(double2), hipMemcpyHostToDevice)) != hipSuccess)
        return fail(e, "copy");
    {
        // wt[q2][p1] = W64^(p1 q2): the pass-2 twiddles of gl_iter_wave_kernel
        std::vector<double2> wt(64);
        for (int q2 = 0; q2 < 16; ++q2)
            for (int p1 = 0; p1 < 4; ++p1) {
                const double a2 = 2.0 * M_PI * (double)(p1 * q2) / 64.0;
                wt[q2 * 4 + p1] = double2{std::cos(a2), -std::sin(a2)};
            }
        if ((e = hipMalloc(&g->wt, wt.size() * sizeof(double2))) != hipSuccess) return fail(e, "hipMalloc");
        if ((e = hipMemcpy(g->wt, wt.data(), wt.size() * sizeof(double2), hipMemcpyHostToDevice)) != hipSuccess)
            return fail(e, "copy");
        // window cosine seeds (c_0, c_1), c_r = cos(2 pi (s + 128 r - woff) / win), at the first sample
        // of each lane: input order (s = 2 L + e), output order (s = 2 (16 (L & 3) + (L >> 2)) + e)
        std::vector<double2> wc(4 * 64);
        for (int L = 0; L < 64; ++L)
            for (int e = 0; e < 2; ++e) {
                const int si = 2 * L + e, so = 2 * (16 * (L & 3) + (L >> 2)) + e;
                const double ai = 2.0 * M_PI * (double)(si - g->g.woff) / cfg->win_length;
                const double ao = 2.0 * M_PI * (double)(so - g->g.woff) / cfg->win_length;
                const double ar = 2.0 * M_PI * 128.0 / cfg->win_length;
                wc[e * 64 + L] = double2{std::cos(ai), std::cos(ai + ar)};
                wc[(2 + e) * 64 + L] = double2{std::cos(ao), std::cos(ao + ar)};
            }
        g->wrot = 2.0 * std::cos(2.0 * M_PI * 128.0 / cfg->win_length);
        if ((e = hipMalloc(&g->winc, wc.size() * sizeof(double2))) != hipSuccess) return fail(e, "hipMalloc");
        if ((e = hipMemcpy(g->winc, wc.data(), wc.size() * sizeof(double2), hipMemcpyHostToDevice)) != hipSuccess)
            return fail(e, "copy");
        g->wave = !getenv_off("TTS_GL_WAVE");
        // window sum-square of a sample q (u = q - woff) with every contributor present: frames
        // i = ceil((u - win + 1) / hop) .. floor(u / hop) in index order, float32 additions of the
        // float64 win^2 as ola_sample makes them; depends on u mod hop only
        const int hop = cfg->hop_length, wl = cfg->win_length;
        std::vector<float> wp(hop);
        for (int r = 0; r < hop; ++r) {
            const int u = r + hop * (wl / hop + 1);
            const int ilo = (u - wl + 1 + hop - 1) / hop, ihi = u / hop;
            float w = 0.f;
            for (int i = ilo; i <= ihi; ++i) w = (float)((double)w + win2[g->g.woff + u - i * hop]);
            wp[r] = w;
        }
        if ((e = hipMalloc(&g->wssp, hop * sizeof(float))) != hipSuccess) return fail(e, "hipMalloc");
        if ((e = hipMemcpy(g->wssp, wp.data(), hop * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess)
            return fail(e, "copy");
    }
    if (inv_mel_basis) {
        const size_t n = (size_t)NB * cfg->num_mels;
        if ((e = hipMalloc(&g->pinv, n * 8)) != hipSuccess) return fail(e, "hipMalloc");
        std::vector<double> pt(n);
        for (int k = 0; k < NB; ++k)
            for (int m = 0; m < cfg->num_mels; ++m) pt[(size_t)m * NB + k] = inv_mel_basis[(size_t)k * cfg->num_mels + m];
        if ((e = hipMemcpy(g->pinv, pt.data(), n * 8, hipMemcpyHostToDevice)) != hipSuccess) return fail(e, "copy");
    }
    // persistent GL loop: status word, timeout (50 ms per wait); needs >= 256 compute units
    {
        int dev = 0, ncu = 0, rate_khz = 0;
        if ((e = hipMalloc(&g->pstatus, 16)) != hipSuccess) return fail(e, "hipMalloc");
        // (an empty speculative run leaves the word as it is: it must start out clean)
        if ((e = hipMemset(g->pstatus, 0, 16)) != hipSuccess) return fail(e, "hipMemset");
        if ((e = hipHostMalloc(reinterpret_cast<void**>(&g->host_status), 2 * sizeof(int), hipHostMallocCoherent)) != hipSuccess)
            return fail(e, "hipHostMalloc");
        // host_status[1] is polled for ++seq (from 1): a recycled pinned block may hold a stale match
        g->host_status[0] = 0;
        g->host_status[1] = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu >= 256 &&
            hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && rate_khz > 0)
            g->tmo = (long long)rate_khz * 50;
        // tests only: a tiny per-wait budget forces the timeout path (status, NaN-poisoned signal)
        const char* tk = getenv("TTS_GL_WAIT_TICKS");
        if (tk && tk[0] && g->tmo > 0) g->tmo = std::max(1LL, atoll(tk));
    }
    *out = g;
    return TTS_OK;
}

}  // extern "C"

namespace tts {
void gl_set_pipeline(tts_gl* g, bool on) { g->pipeline = on; }

// small batches fuse the overlap-add into the iteration launch; at most 256 frames in all run the
// whole loop as one persistent launch (host values only)
static bool gl_fused_path(const tts_gl* g, int B, int Fmax) {
    const char* fz = getenv("TTS_GL_FUSED");
    return ((int64_t)B * Fmax <= 1024 || (fz && fz[0] == '1')) && (g->g.win + g->g.hop - 1) / g->g.hop <= OLA_MAX;
}
// The persistent loop overwrites a frame's ping-pong slot once its own contributors have moved on:
// safe when every reader of a frame is one of its contributors.  Frame f reads the signal at the
// reflected positions R(W_f), W_f = [f hop - win/2, f hop + win/2) (centred STFT frames), and its
// contributors are the frames fi whose windows W_fi hold one of them.  While one reflection
// suffices (win/2 < hop (F - 1)), R maps the part of W_f outside [0, N) into W_f's own part inside,
// so R(W_f) = W_f n [0, N) and "f reads fi" <=> W_f n W_fi n [0, N) != {} is symmetric.  Shorter
// sentences are checked by brute force (host copy of the kernels' index maps).
static int reflect_host(int p, int N) {
    if ((unsigned)p < (unsigned)N) return p;
    if (N == 1) return 0;
    const int period = 2 * (N - 1);
    int pp = p % period;
    if (pp < 0) pp += period;
    return pp < N ? pp : period - pp;
}
static bool contrib_symmetric(const Geo& g, int F) {
    if (2 * g.hop * (F - 1) > g.win + 2) return true;
    const int N = g.hop * (F - 1);
    std::vector<char> c((size_t)F * F, 0);
    for (int f = 0; f < F; ++f)
        for (int n = g.woff; n < g.woff + g.win; ++n) {
            const int q = reflect_host(f * g.hop + n - NFFT / 2, N) + NFFT / 2;
            if (q < g.woff) continue;
            int ilo = q - g.woff - g.win + 1;
            ilo = ilo <= 0 ? 0 : (ilo + g.hop - 1) / g.hop;
            const int ihi = std::min((q - g.woff) / g.hop, F - 1);
            for (int fi = ilo; fi <= ihi; ++fi) c[(size_t)f * F + fi] = 1;
        }
    for (int f = 0; f < F; ++f)
        for (int fi = 0; fi < F; ++fi)
            if (c[(size_t)f * F + fi] != c[(size_t)fi * F + f]) return false;
    return true;
}
// The persistent loop's gather layout for a sentence of F frames (gl_persistent_kernel): every
// overlap-add contributor within GL_DMAX frames and at most GL_PAIRS granule pairs per thread.  Only
// frames whose STFT window reaches a sentence edge (reflection) differ from the interior ones: those
// and one interior frame are checked, restating the kernel's index arithmetic.
static bool gather_fits(const Geo& g, int F) {
    const int N = g.hop * (F - 1);
    auto frame_ok = [&](int f) {
        int lo[GL_SLOTS], hi[GL_SLOTS];
        for (int k = 0; k < GL_SLOTS; ++k) {
            lo[k] = 1 << 30;
            hi[k] = -1;
        }
        for (int n = g.woff; n < g.woff + g.win; ++n) {
            const int q = reflect_host(f * g.hop + n - NFFT / 2, N) + NFFT / 2;
            if (q < g.woff) continue;
            int ilo = q - g.woff - g.win + 1;
            ilo = ilo <= 0 ? 0 : (ilo + g.hop - 1) / g.hop;
            const int ihi = std::min((q - g.woff) / g.hop, F - 1);
            for (int fi = ilo; fi <= ihi; ++fi) {
                const int sl = fi - f + GL_DMAX;
                if (sl < 0 || sl >= GL_SLOTS || fi - ilo >= OLA_MAX) return false;
                lo[sl] = std::min(lo[sl], q - fi * g.hop - g.fb);
                hi[sl] = std::max(hi[sl], q - fi * g.hop - g.fb);
            }
        }
        int pairs = 0;
        for (int k = 0; k < GL_SLOTS; ++k)
            if (hi[k] >= 0) pairs += (hi[k] - (lo[k] & ~1)) / 2 + 1;
        return pairs <= GL_PAIRS * GL_THREADS;
    };
    bool interior_done = false;
    for (int f = 0; f < F; ++f) {
        const bool edge = f * g.hop + g.woff - NFFT / 2 < 0 || f * g.hop + g.woff + g.win - 1 - NFFT / 2 >= N;
        if (!edge && interior_done) continue;
        if (!frame_ok(f)) return false;
        if (!edge) interior_done = true;
    }
    return (g.winp % 2) == 0;
}

bool gl_persistent_path(tts_gl* g, int B, int Fmax, int frames_total, int iters) {
    // (tags hold the iteration in 14 bits below the salt)
    if (!(gl_fused_path(g, B, Fmax) && iters > 0 && iters < (1 << 14) && frames_total <= 512 && g->tmo > 0 &&
          !getenv_off("TTS_RESIDENT")))
        return false;
    // every frame count the run may have (a speculative run knows only the upper bound Fmax)
    for (int F = 2; F <= Fmax; ++F) {
        if (2 * g->g.hop * (F - 1) > g->g.win + 2) break;  // symmetric from here on (above)
        if (!contrib_symmetric(g->g, F)) return false;
    }
    if ((int)g->gather_fit.size() <= Fmax) g->gather_fit.resize(Fmax + 1, -1);
    for (int F = 2; F <= Fmax; ++F) {
        if (g->gather_fit[F] < 0) g->gather_fit[F] = gather_fits(g->g, F) ? 1 : 0;
        if (!g->gather_fit[F]) return false;
    }
    return true;
}

// numpy-stream phases for a run of B sentences (F_dev on the device, read on s) into `out`
// ([B][1025][Fmax]), continuing the handle's MT19937 state; draws on another stream than the last
// one wait for it (the stream's order is the draws' order)
static tts_status mt_draw(tts_gl* g, const int* F_dev, int B, int Fmax, double* out, hipStream_t s) {
    TTS_CHECK(B <= MT_MAX_BATCH, TTS_ERR_UNSUPPORTED, "numpy-stream phases: at most 1024 sentences per run");
    if (g->mt_stream && g->mt_stream != s) TTS_HIP(hipStreamWaitEvent(s, g->ev_mt, 0));
    TTS_HIP(mt_draw_phases(g->mt_state, F_dev, B, Fmax, out, &g->mt_work, s));
    TTS_HIP(hipEventRecord(g->ev_mt, s));
    g->mt_stream = s;
    return TTS_OK;
}

tts_status gl_collect(tts_gl* g) {
    if (!g->pending) return TTS_OK;
    g->pending = false;
    if (g->last_timed) {
        TTS_HIP(hipEventSynchronize(g->ev_done));
        TTS_HIP(hipEventElapsedTime(&g->last_ms, g->ev_t0, g->ev_t1));
    } else if (g->last_persistent) {
        // pipeline mode: no event markers; the overlap-add launch set the status, then the sequence
        TTS_HIP(spin_word(g->host_status + 1, g->seq, g->seq_stream));
    }
    if (g->last_persistent)
        TTS_CHECK(g->host_status[0] == 0, TTS_ERR_HIP, "persistent Griffin-Lim: a hand-off wait timed out (internal error)");
    return TTS_OK;
}
}  // namespace tts

extern "C" {

tts_status tts_gl_run(tts_gl* g, int mode, const float* spec, const int32_t* F, int B, int Fmax,
                      const double* phase_u, uint64_t seed, int iters, double* wav, void* stream) {
    return tts::gl_run_dev(g, mode, spec, F, nullptr, B, Fmax, phase_u, seed, iters, wav, static_cast<hipStream_t>(stream));
}

tts_status tts_gl_set_phase_state(tts_gl* g, const uint32_t* key, int pos) {
    TTS_CHECK(g, TTS_ERR_INVALID, "null handle");
    if (!key) {
        g->mt_armed = false;
        return TTS_OK;
    }
    TTS_CHECK(pos >= 0 && pos <= 624, TTS_ERR_INVALID, "MT19937 position must be in [0, 624]");
    if (!g->mt_state) TTS_HIP(hipMalloc(&g->mt_state, 625 * sizeof(unsigned)));
    if (g->mt_stream) TTS_HIP(hipEventSynchronize(g->ev_mt));  // a draw may still read the old state
    unsigned h[625];
    std::copy(key, key + 624, h);
    h[624] = (unsigned)pos;
    TTS_HIP(hipMemcpy(g->mt_state, h, sizeof(h), hipMemcpyHostToDevice));
    g->mt_armed = true;
    return TTS_OK;
}

tts_status tts_gl_get_phase_state(tts_gl* g, uint32_t* key, int* pos) {
    TTS_CHECK(g && key && pos, TTS_ERR_INVALID, "null argument");
    TTS_CHECK(g->mt_state, TTS_ERR_INVALID, "no phase state set (tts_gl_set_phase_state)");
    if (g->mt_stream) TTS_HIP(hipEventSynchronize(g->ev_mt));
    unsigned h[625];
    TTS_HIP(hipMemcpy(h, g->mt_state, sizeof(h), hipMemcpyDeviceToHost));
    std::copy(h, h + 624, key);
    *pos = (int)h[624];
    return TTS_OK;
}

tts_status tts_gl_draw_phases(tts_gl* g, const int32_t* F, int B, int Fmax, double* phase_u, void* stream) {
    TTS_CHECK(g && F && phase_u && B >= 1 && Fmax >= 1, TTS_ERR_INVALID, "bad draw_phases arguments");
    TTS_CHECK(g->mt_armed, TTS_ERR_INVALID, "no phase state set (tts_gl_set_phase_state)");
    for (int b = 0; b < B; ++b) TTS_CHECK(F[b] >= 0 && F[b] <= Fmax, TTS_ERR_INVALID, "F[b] out of range [0, Fmax]");
    hipStream_t s = static_cast<hipStream_t>(stream);
    // (mt_F is rewritten below: a draw on another stream may still read it)
    if (g->mt_stream && g->mt_stream != s) TTS_HIP(hipStreamWaitEvent(s, g->ev_mt, 0));
    if (B > g->mt_F_n) {
        if (g->mt_stream) TTS_HIP(hipEventSynchronize(g->ev_mt));
        if (g->mt_F) TTS_HIP(hipFree(g->mt_F));
        g->mt_F = nullptr;
        TTS_HIP(hipMalloc(&g->mt_F, B * sizeof(int)));
        g->mt_F_n = B;
    }
    TTS_HIP(hipMemcpyAsync(g->mt_F, F, B * sizeof(int), hipMemcpyHostToDevice, s));
    return tts::mt_draw(g, g->mt_F, B, Fmax, phase_u, s);
}

tts_status tts_gl_save_pcm16(tts_gl* g, const double* wav, int64_t pitch, const int64_t* n, int B, int gap,
                             double peak, int16_t* out, void* stream) {
    TTS_CHECK(g && wav && n && out && B >= 1 && gap >= 0, TTS_ERR_INVALID, "bad save_pcm16 arguments");
    hipStream_t s = static_cast<hipStream_t>(stream);
    for (int b = 0; b < B; ++b) TTS_CHECK(n[b] >= 0 && n[b] <= pitch, TTS_ERR_INVALID, "n[b] out of range [0, pitch]");
    if (!g->pcm_peak) TTS_HIP(hipMalloc(&g->pcm_peak, sizeof(unsigned long long)));
    if (B + 1 > g->pcm_start_n) {
        TTS_HIP(hipStreamSynchronize(s));  // (the previous join on this stream may still read it)
        if (g->pcm_start) TTS_HIP(hipFree(g->pcm_start));
        g->pcm_start = nullptr;
        TTS_HIP(hipMalloc(&g->pcm_start, (B + 1) * sizeof(int64_t)));
        g->pcm_start_n = B + 1;
    }
    g->pcm_start_h.assign(B + 1, 0);
    for (int b = 0; b < B; ++b) g->pcm_start_h[b + 1] = g->pcm_start_h[b] + n[b] + gap;
    TTS_HIP(hipMemcpyAsync(g->pcm_start, g->pcm_start_h.data(), (B + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    TTS_HIP(tts::pcm16_join(wav, pitch, g->pcm_start, g->pcm_start_h[B], B, gap, peak, g->pcm_peak, out, s));
    return TTS_OK;
}
}  // extern "C"

namespace tts {
// tts_gl_run, optionally with the frame counts also on the device (F_dev, the same values as F:
// tts_synth_run passes the decoder's step counts at r = 1): the persistent loop's launches then
// read them there and the upload is skipped (the graph-replayed fallbacks still upload into the
// handle's own array, which their graphs bake in).  F_bound: F holds only upper bounds of the
// device counts (a run enqueued before the decoder's step counts reach the host, same stream):
// the fallbacks then copy F_dev into the handle's array on the device.
tts_status gl_run_dev(tts_gl* g, int mode, const float* spec, const int32_t* F, const int* F_dev, int B, int Fmax,
                      const double* phase_u, uint64_t seed, int iters, double* wav, hipStream_t stream, bool F_bound) {
    TTS_CHECK(g && spec && F && wav && B >= 1 && Fmax >= 2 && iters >= 0, TTS_ERR_INVALID, "bad gl_run arguments");
    TTS_CHECK(!F_bound || F_dev, TTS_ERR_INVALID, "F_bound needs device frame counts");
    TTS_CHECK(mode == TTS_GL_FROM_MEL || mode == TTS_GL_FROM_LINEAR, TTS_ERR_INVALID, "bad mode");
    TTS_CHECK(mode == TTS_GL_FROM_LINEAR || g->pinv, TTS_ERR_INVALID, "mel mode needs inv_mel_basis at create");
    for (int b = 0; b < B; ++b) TTS_CHECK(F[b] >= 2 && F[b] <= Fmax, TTS_ERR_INVALID, "F[b] out of range [2, Fmax]");
    hipStream_t cs = stream;
    hipStream_t s = g->pipeline ? cs : g->stream;
    const Geo geo = g->g;
    const int64_t Nmax = (int64_t)geo.hop * (Fmax - 1);
    {
        tts_status pst = gl_collect(g);  // the previous pipeline run, if any (its status, timing)
        if (pst) return pst;
    }
    // workspace (grow only; graphs bake the buffer addresses and are dropped when they move)
    const size_t needS = (size_t)B * Fmax * NB, needF = (size_t)2 * B * Fmax * geo.winp, needY = (size_t)B * Nmax;
    bool moved = false;
    auto grow = [&](void** p, size_t& have, size_t need, size_t elem) -> tts_status {
        if (need <= have) return TTS_OK;
        if (*p) TTS_HIP(hipFree(*p));
        *p = nullptr;
        TTS_HIP(hipMalloc(p, need * elem));
        have = need;
        moved = true;
        return TTS_OK;
    };
    // the workspace may move below: nothing of this handle may still be in flight (a pipeline
    // run's stream has been synchronised by its caller before the next run)
    if (!g->pipeline) TTS_HIP(hipStreamSynchronize(s));
    tts_status st;
    if ((st = grow(reinterpret_cast<void**>(&g->S), g->S_n, needS, sizeof(spec_t)))) return st;
    if ((st = grow(reinterpret_cast<void**>(&g->frames), g->fr_n, needF, sizeof(frame_t)))) return st;
    if ((st = grow(reinterpret_cast<void**>(&g->y), g->y_n, needY, 4))) return st;
    if (B > g->Fcap_B) {
        if (g->F) TTS_HIP(hipFree(g->F));
        g->F = nullptr;
        TTS_HIP(hipMalloc(&g->F, B * sizeof(int)));
        g->Fcap_B = B;
        moved = true;
    }
    if (moved) {
        for (auto& kv : g->graphs) (void)hipGraphExecDestroy(kv.second);
        g->graphs.clear();
    }
    if (s != cs) {
        TTS_HIP(hipEventRecord(g->ev_in, cs));
        TTS_HIP(hipStreamWaitEvent(s, g->ev_in, 0));
    }
    // path choice (host values only): small batches fuse the overlap-add into the iteration launch;
    // at most 512 frames in all run the whole loop as one persistent launch
    const char* fz = getenv("TTS_GL_FUSED");
    const bool fused = gl_fused_path(g, B, Fmax);
    int frames_total = 0;
    for (int b = 0; b < B; ++b) frames_total += F[b];
    const bool persistent = gl_persistent_path(g, B, Fmax, frames_total, iters);
    // the launches read the frame counts from F_dev when the persistent loop takes them all; the
    // graph-replayed loops read the handle's own array, filled from F_dev when there is one (a
    // speculative run's host F is only an upper bound: tts_synth_run)
    const int* Fd = persistent && F_dev ? F_dev : g->F;  // (reassigned if the persistent launch falls back)
    if (Fd == g->F) {
        if (F_bound) TTS_HIP(hipMemcpyAsync(g->F, F_dev, B * sizeof(int), hipMemcpyDeviceToDevice, s));
        else TTS_HIP(hipMemcpyAsync(g->F, F, B * sizeof(int), hipMemcpyHostToDevice, s));
    }
    if (!phase_u && g->mt_armed) {
        // the reference's np.random.rand draws, continued on the device from numpy's state
        // (tts_gl_set_phase_state): one [1025][F_b] draw per sentence in batch order
        const size_t needP = (size_t)B * NB * Fmax;
        if (needP > g->mt_phase_n) {
            if (g->mt_stream) TTS_HIP(hipStreamSynchronize(g->mt_stream));  // an earlier run may still read it
            if (g->mt_phase) TTS_HIP(hipFree(g->mt_phase));
            g->mt_phase = nullptr;
            TTS_HIP(hipMalloc(&g->mt_phase, needP * sizeof(double)));
            g->mt_phase_n = needP;
        }
        if ((st = mt_draw(g, Fd, B, Fmax, g->mt_phase, s))) return st;
        phase_u = g->mt_phase;
    }
    MagArgs ma{};
    ma.mode = mode;
    ma.spec = spec;
    ma.n_in = mode == TTS_GL_FROM_MEL ? g->cfg.num_mels : NB;
    ma.Fmax = Fmax;
    ma.F = Fd;
    ma.pinv = g->pinv;
    ma.S = g->S;
    ma.min_db = g->cfg.min_level_db;
    ma.ref_db = g->cfg.ref_level_db;
    ma.power = g->cfg.power;
    ma.max_norm = g->cfg.max_norm;
    ma.signal_norm = g->cfg.signal_norm;
    ma.symmetric = g->cfg.symmetric_norm;
    ma.clip = g->cfg.clip_norm;
    if (mode == TTS_GL_FROM_LINEAR)
        hipLaunchKernelGGL(gl_linear_magnitude_kernel,
                           dim3((unsigned)(((int64_t)Fmax * NB + 256 * LIN_PER - 1) / (256 * LIN_PER)), B), dim3(256), 0, s,
                           ma);
    else
        hipLaunchKernelGGL(gl_magnitude_kernel, dim3((NB + MAG_KT - 1) / MAG_KT, (Fmax + MAG_FT - 1) / MAG_FT, B),
                           dim3(256), 0, s, ma);
    TTS_HIP(hipGetLastError());
    const size_t fstride = (size_t)B * Fmax * geo.winp;
    // the persistent loop reads and writes two slots of tagged granules (gl_persistent_kernel);
    // the other loops two slots of float32 frames (TTS_GL_FUSED=1 forces the fused form at any
    // batch: measurement knob)
    if (persistent && 2 * fstride > g->pgr_n) {
        if (g->pgr) TTS_HIP(hipFree(g->pgr));
        g->pgr = nullptr;
        TTS_HIP(hipMalloc(&g->pgr, 2 * fstride * sizeof(gran_t)));
        g->pgr_n = 2 * fstride;
        // fresh memory may hold a freed handle's granules, and every handle's salts start at 1: a
        // stale granule there can carry a tag this handle is about to wait for.  Filled with a word
        // that is no live tag and not 0 (0 marks an absent contributor: gl_persistent_kernel)
        TTS_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(g->pgr), GL_GRAN_FILL, g->pgr_n * 2, s));
    }
    // frame slot i of the two ping-pong slots of the fused / batched loops
    auto slot = [&](int i) -> void* { return static_cast<frame_t*>(g->frames) + (i & 1) * fstride; };
    if (persistent) {  // the initial iSTFT tags its granules with the launch's salt
        g->salt = (g->salt + 1) & 0x3FFFF;
        if (g->salt == 0) {
            // wrapped: a granule of the launch 2^18 back could carry a current tag
            g->salt = 1;
            TTS_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(g->pgr), GL_GRAN_FILL, g->pgr_n * 2, s));
        }
    }
    IterArgs ia{};
    ia.S = g->S;
    ia.F = Fd;
    ia.Fmax = Fmax;
    ia.B = B;
    ia.g = geo;
    ia.c = GLConst{g->win, g->win2, g->tw};
    ia.phase_u = phase_u;
    ia.seed = seed;
    ia.y = g->y;
    ia.Nmax = Nmax;
    ia.next = persistent ? static_cast<void*>(g->pgr) : slot(0);
    ia.wt = g->wt;
    ia.winc = g->winc;
    ia.wrot = g->wrot;
    ia.gtag = g->salt << 14;
    if (persistent) {
        if ((size_t)B * Fmax > g->flags_n) {
            if (g->flags) TTS_HIP(hipFree(g->flags));
            g->flags = nullptr;
            TTS_HIP(hipMalloc(&g->flags, sizeof(unsigned) * (size_t)B * Fmax));
            g->flags_n = (size_t)B * Fmax;
        }
        // table entries are salted per launch, and a new handle can get a freed one's words: the
        // initial iSTFT launch zeroes them and the status word
        ia.zero_flags = g->flags;
        ia.zero_status = g->pstatus;
    }
    const dim3 grid(Fmax, B), block(GL_THREADS);
    static const bool wave_init = [] {  // measurement: TTS_GL_WAVE_INIT=0 keeps the block-kernel init
        const char* v = getenv("TTS_GL_WAVE_INIT");
        return !(v && v[0] == '0');
    }();
    if (persistent) hipLaunchKernelGGL((gl_iter_kernel<true, false, gran_t>), grid, block, 0, s, ia);
    else if (!fused && g->wave && wave_init)  // the batched loop's own layout for its first launch
        hipLaunchKernelGGL(gl_iter_wave_kernel<true>, grid, dim3(64), 0, s, ia);
    else hipLaunchKernelGGL((gl_iter_kernel<true, false, frame_t>), grid, block, 0, s, ia);
    ia.zero_flags = nullptr;
    ia.zero_status = nullptr;
    TTS_HIP(hipGetLastError());
    // loop timers and the completion event outside pipeline mode only (each event marker holds the
    // GPU ~5.8 us between the kernels around it); a pipeline run's status travels by sequence word
    const bool timed = !g->pipeline;
    if (timed) TTS_HIP(hipEventRecord(g->ev_t0, s));
    FinArgs fa{};
    fa.F = Fd;
    fa.Fmax = Fmax;
    fa.B = B;
    fa.g = geo;
    fa.c = ia.c;
    fa.y = g->y;
    fa.Nmax = Nmax;
    fa.wssp = g->wssp;
    const dim3 ogrid((Nmax + 255) / 256, B), oblock(256);
    bool persistent_ran = false;
    if (persistent) {
        PersArgs pa{};
        pa.it = ia;
        pa.frames = g->pgr;
        pa.fstride = (int64_t)fstride;
        pa.iters = iters;
        pa.xtab = g->flags;
        pa.salt = g->salt;
        pa.tmo = g->tmo;
        pa.status = g->pstatus;
        pa.drop_f = -1;
        if (const char* inj = getenv("TTS_GL_INJECT_DROP"); inj && inj[0]) pa.drop_f = atoi(inj);
        static const bool gl_nowait = [] {
            const char* v = getenv("TTS_GL_NOWAIT");
            return v && v[0] == '1';
        }();
        pa.nowait = gl_nowait;
        static const int gl_first_sleep = [] {
            const char* v = getenv("TTS_GL_FIRST_SLEEP");
            return v ? atoi(v) : 4;  // round 6: -19 us per configs[1] sentence (tools/cases_sleep.txt)
        }();
        pa.first_sleep = gl_first_sleep;
        long long* prof = nullptr;
        const char* phases = getenv("TTS_GL_PHASES");
        if (phases && phases[0]) {  // diagnostic: phase ticks of frame TTS_GL_PHASES (stderr)
            TTS_HIP(hipMalloc(&prof, 6 * sizeof(long long)));
            TTS_HIP(hipMemsetAsync(prof, 0, 6 * sizeof(long long), s));
            pa.prof = prof;
            pa.prof_f = std::min(atoi(phases), frames_total - 1);
        }
        // every workgroup waits on its neighbours inside the launch: co-residency guaranteed, or
        // nothing runs and the fused loop below takes the iterations (bitwise the same waveform)
        void* kargs[] = {&pa};
        // dynamic LDS: the gather buffer, GL_SLOTS frame slots + the zero word
        const size_t og_bytes = ((size_t)GL_SLOTS * geo.winp + 2) * sizeof(float);
        // up to 256 workgroups: one per compute unit; up to 512: two per compute unit (gl_persistent2_kernel)
        const bool two = (long long)grid.x * grid.y > 256;
        const void* pfn = two ? reinterpret_cast<const void*>(&gl_persistent2_kernel)
                              : reinterpret_cast<const void*>(&gl_persistent_kernel);
        static const hipError_t attr = [] {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gl_persistent_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
            if (e == hipSuccess)
                e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gl_persistent2_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
            return e;
        }();
        TTS_HIP(attr);
        TTS_CHECK(og_bytes <= 96 * 1024, TTS_ERR_INVALID, "persistent Griffin-Lim: window too long for the gather buffer");
        TTS_HIP(launch_persistent(pfn, grid, block, kargs, og_bytes, s, &persistent_ran));
        if (!persistent_ran) {
            // the initial iSTFT wrote slot 0 of the granule buffer: hand it to the fused loop
            hipLaunchKernelGGL(gl_gran_to_frames_kernel, dim3((unsigned)((fstride + 255) / 256)), dim3(256), 0, s,
                               g->pgr, static_cast<frame_t*>(g->frames), (int64_t)fstride);
            TTS_HIP(hipGetLastError());
            if (prof) {
                TTS_HIP(hipStreamSynchronize(s));
                TTS_HIP(hipFree(prof));
                prof = nullptr;
            }
        }
        if (prof) {
            long long h[6];
            TTS_HIP(hipMemcpyAsync(h, prof, sizeof(h), hipMemcpyDeviceToHost, s));
            TTS_HIP(hipStreamSynchronize(s));
            TTS_HIP(hipFree(prof));
            int rate_khz = 100000, dev = 0;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev);
            static const char* names[6] = {"gather", "ola_sums", "fwd_fft", "spectrum", "inv_fft", "store"};
            fprintf(stderr, "TTS_GL_PHASES frame %d, us per iteration:", pa.prof_f);
            for (int k = 0; k < 6; ++k) fprintf(stderr, " %s %.3f", names[k], h[k] * 1e3 / rate_khz / iters);
            fprintf(stderr, "\n");
        }
    }
    if (!persistent_ran && Fd != g->F) {
        // the persistent loop could not be placed: its fallbacks replay graphs that bake the
        // handle's own frame-count array in
        if (F_bound) TTS_HIP(hipMemcpyAsync(g->F, F_dev, B * sizeof(int), hipMemcpyDeviceToDevice, s));
        else TTS_HIP(hipMemcpyAsync(g->F, F, B * sizeof(int), hipMemcpyHostToDevice, s));
        Fd = g->F;
        ia.F = fa.F = Fd;
    }
    if (!persistent_ran && iters > 0) {
        // one iteration = overlap-add of the previous frames into the float32 signal (every
        // sample once) + one workgroup per frame for STFT -> phase -> iSTFT of that signal
        GraphKey key{B, Fmax, iters};
        auto it = g->graphs.find(key);
        if (it == g->graphs.end()) {
            hipGraph_t graph = nullptr;
            TTS_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            for (int i = 0; i < iters; ++i) {
                IterArgs a = ia;
                a.phase_u = nullptr;
                a.next = slot(i + 1);
                if (fused) {
                    a.prev = slot(i);
                    hipLaunchKernelGGL((gl_iter_kernel<false, true, frame_t>), grid, block, 0, s, a);
                } else {
                    FinArgs o = fa;
                    o.frames = slot(i);
                    launch_ola_frames(o, s);
                    if (g->wave)
                        hipLaunchKernelGGL(gl_iter_wave_kernel<false>, grid, dim3(64), 0, s, a);
                    else
                        hipLaunchKernelGGL((gl_iter_kernel<false, false, frame_t>), grid, block, 0, s, a);
                }
            }
            hipError_t ce = hipGetLastError();
            hipError_t ee = hipStreamEndCapture(s, &graph);
            TTS_HIP(ce);
            TTS_HIP(ee);
            hipGraphExec_t exec = nullptr;
            TTS_HIP(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
            TTS_HIP(hipGraphDestroy(graph));
            it = g->graphs.emplace(key, exec).first;
        }
        TTS_HIP(hipGraphLaunch(it->second, s));
    }
    if (timed) TTS_HIP(hipEventRecord(g->ev_t1, s));
    fa.frames = persistent_ran ? static_cast<void*>(g->pgr + (size_t)(iters & 1) * fstride) : slot(iters);
    fa.status = persistent_ran ? g->pstatus : nullptr;
    fa.host_status = persistent_ran ? g->host_status : nullptr;  // (no read-back copy launch)
    if (persistent_ran && !timed) {
        fa.host_seq = g->host_status + 1;
        fa.seq = ++g->seq;
        g->seq_stream = s;
    }
    if (persistent_ran) hipLaunchKernelGGL(gl_ola_kernel<gran_t>, ogrid, oblock, 0, s, fa);
    else launch_ola_frames(fa, s);
    fa.status = nullptr;
    fa.host_status = nullptr;
    fa.host_seq = nullptr;
    TTS_HIP(hipGetLastError());
    {
        // de-emphasis chunks: each starts `look` samples early, |c|^look <= 1e-22; one chunk per
        // sentence (look 0) when that does not fit one scan tile
        const double c = g->cfg.preemphasis, ac = std::fabs(c);
        int64_t chunk = SCAN_CHUNK, look = 0;
        if (ac > 0.0) {
            const double need = ac < 1.0 ? std::ceil(std::log(1e-22) / std::log(ac)) : 1e30;
            if (need <= (double)(SCAN_THREADS * SCAN_PER - SCAN_CHUNK - 8)) look = (int64_t)need;
            else chunk = Nmax;
        }
        const dim3 sgrid((unsigned)((Nmax + chunk - 1) / chunk), B);
        hipLaunchKernelGGL(preemph_scan_kernel, sgrid, dim3(SCAN_THREADS), 0, s, g->y, Nmax, Fd, geo.hop, c,
                           c != 0.0 ? 1 : 0, chunk, look, wav);
    }
    TTS_HIP(hipGetLastError());
    g->last_persistent = persistent_ran;
    g->last_path = persistent_ran ? TTS_GL_PATH_PERSISTENT : fused ? TTS_GL_PATH_FUSED : TTS_GL_PATH_UNFUSED;
    g->last_launches = persistent_ran ? 1 : (fused ? 1 : 2) * iters;
    if (timed) {
        TTS_HIP(hipEventRecord(g->ev_done, s));
        if (s != cs) TTS_HIP(hipStreamWaitEvent(cs, g->ev_done, 0));
    } else {
        g->last_ms = 0.f;  // (pipeline mode: not timed)
    }
    g->last_timed = timed;
    g->pending = true;
    if (!g->pipeline) {
        tts_status cst = gl_collect(g);
        if (cst) return cst;
    }
    g->last_fused = fused;
    g->have_last = true;
    g->last_iter = ia;
    g->last_fin = fa;
    g->last_fstride = fstride;
    return TTS_OK;
}

}  // namespace tts

extern "C" {

tts_status tts_gl_profile(tts_gl* g, int reps, float* kernel_ms, int n_kernels) {
    TTS_CHECK(g && kernel_ms && n_kernels >= TTS_GL_KERNELS && reps >= 1, TTS_ERR_INVALID, "bad profile arguments");
    TTS_CHECK(g->have_last, TTS_ERR_INVALID, "tts_gl_profile needs a previous tts_gl_run");
    {
        tts_status pst = gl_collect(g);
        if (pst) return pst;
    }
    hipStream_t s = g->stream;
    hipEvent_t ev[3];
    for (auto& e : ev) TTS_HIP(hipEventCreate(&e));
    const IterArgs& ia = g->last_iter;
    const dim3 grid(ia.Fmax, ia.B), block(GL_THREADS);
    double it_ms = 0.0, ola_ms = 0.0;
    for (int r = 0; r < reps; ++r) {
        // one GL iteration as tts_gl_run launches it: overlap-add -> per-frame STFT/iSTFT
        FinArgs f = g->last_fin;
        const size_t es = sizeof(frame_t);
        f.frames = static_cast<char*>(g->frames) + (r & 1) * g->last_fstride * es;
        IterArgs a = ia;
        a.phase_u = nullptr;
        a.next = static_cast<char*>(g->frames) + ((r + 1) & 1) * g->last_fstride * es;
        a.prev = f.frames;
        TTS_HIP(hipEventRecord(ev[0], s));
        if (!g->last_fused)
            launch_ola_frames(f, s);
        TTS_HIP(hipGetLastError());
        TTS_HIP(hipEventRecord(ev[1], s));
        if (g->last_fused)
            hipLaunchKernelGGL((gl_iter_kernel<false, true, frame_t>), grid, block, 0, s, a);
        else if (g->wave)
            hipLaunchKernelGGL(gl_iter_wave_kernel<false>, grid, dim3(64), 0, s, a);
        else
            hipLaunchKernelGGL((gl_iter_kernel<false, false, frame_t>), grid, block, 0, s, a);
        TTS_HIP(hipGetLastError());
        TTS_HIP(hipEventRecord(ev[2], s));
        TTS_HIP(hipEventSynchronize(ev[2]));
        float a_ms = 0.f, b_ms = 0.f;
        TTS_HIP(hipEventElapsedTime(&b_ms, ev[0], ev[1]));
        TTS_HIP(hipEventElapsedTime(&a_ms, ev[1], ev[2]));
        it_ms += a_ms;
        ola_ms += b_ms;
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    kernel_ms[0] = (float)(it_ms / reps);
    kernel_ms[1] = (float)(ola_ms / reps);
    return TTS_OK;
}


tts_status tts_gl_set_mel_basis(tts_gl* g, const double* mel_basis) {
    TTS_CHECK(g && mel_basis, TTS_ERR_INVALID, "null argument");
    const size_t n = (size_t)g->cfg.num_mels * NB;
    if (!g->basis) TTS_HIP(hipMalloc(&g->basis, n * sizeof(double)));
    TTS_HIP(hipMemcpy(g->basis, mel_basis, n * sizeof(double), hipMemcpyHostToDevice));
    return TTS_OK;
}

tts_status tts_gl_melspectrogram(tts_gl* g, const double* wav, const int32_t* N, int B, int64_t Nmax, float* mel,
                                 int Fmax, void* stream) {
    TTS_CHECK(g && wav && N && mel && B >= 1 && Fmax >= 1, TTS_ERR_INVALID, "bad melspectrogram arguments");
    TTS_CHECK(g->basis, TTS_ERR_INVALID, "tts_gl_melspectrogram needs tts_gl_set_mel_basis first");
    for (int b = 0; b < B; ++b) {
        TTS_CHECK(N[b] >= 2 && N[b] <= Nmax, TTS_ERR_INVALID, "N[b] out of range [2, Nmax]");
        TTS_CHECK(1 + N[b] / g->g.hop <= Fmax, TTS_ERR_INVALID, "Fmax < 1 + N[b] / hop");
    }
    hipStream_t cs = static_cast<hipStream_t>(stream);
    hipStream_t s = g->stream;
    if (B > g->NS_cap) {
        TTS_HIP(hipStreamSynchronize(s));
        if (g->NS) TTS_HIP(hipFree(g->NS));
        g->NS = nullptr;
        TTS_HIP(hipMalloc(&g->NS, B * sizeof(int)));
        g->NS_cap = B;
    }
    TTS_HIP(hipEventRecord(g->ev_in, cs));
    TTS_HIP(hipStreamWaitEvent(s, g->ev_in, 0));
    TTS_HIP(hipMemcpyAsync(g->NS, N, B * sizeof(int), hipMemcpyHostToDevice, s));
    TTS_HIP(hipMemsetAsync(mel, 0, sizeof(float) * (size_t)B * Fmax * g->cfg.num_mels, s));
    MelArgs a{};
    a.wav = wav;
    a.Nmax = Nmax;
    a.N = g->NS;
    a.Fmax = Fmax;
    a.g = g->g;
    a.c = GLConst{g->win, g->win2, g->tw};
    a.basis = g->basis;
    a.n_mels = g->cfg.num_mels;
    a.coef = g->cfg.preemphasis;
    a.min_db = g->cfg.min_level_db;
    a.min_level = std::exp((double)g->cfg.min_level_db / 20.0 * std::log(10.0));  // utils/audio.py:122
    a.ref_db = g->cfg.ref_level_db;
    a.max_norm = g->cfg.max_norm;
    a.signal_norm = g->cfg.signal_norm;
    a.symmetric = g->cfg.symmetric_norm;
    a.clip = g->cfg.clip_norm;
    a.mel = mel;
    hipLaunchKernelGGL(mel_analysis_kernel, dim3(Fmax, B), dim3(GL_THREADS), 0, s, a);
    TTS_HIP(hipGetLastError());
    TTS_HIP(hipEventRecord(g->ev_out, s));
    TTS_HIP(hipStreamWaitEvent(cs, g->ev_out, 0));
    return TTS_OK;
}

tts_status tts_gl_last_path(tts_gl* g, int* path) {
    TTS_CHECK(g && path, TTS_ERR_INVALID, "null argument");
    *path = g->last_path;
    return TTS_OK;
}

tts_status tts_gl_last_timing(tts_gl* g, float* loop_ms, int* launches) {
    TTS_CHECK(g && loop_ms && launches, TTS_ERR_INVALID, "null argument");
    {
        tts_status pst = gl_collect(g);
        if (pst) return pst;
    }
    *loop_ms = g->last_ms;
    *launches = g->last_launches;
    return TTS_OK;
}

}  // extern "C"

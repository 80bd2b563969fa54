// Batched Griffin-Lim vocoder (AudioProcessor.inv_mel_spectrogram / inv_spectrogram,
// utils/audio.py:154-201, librosa 0.6.2 stft/istft semantics) for gfx950.
//
// HBM layout (per call):
//   S      [B][Fmax][1025]       |S|^power, frame-major (one 4.1 KB row per frame)
//   frames [2][B][Fmax][WINP]    windowed inverse-FFT output of every frame, window support only
//                                (WIN = 1102 samples; the padded Hann is zero elsewhere)
// One workgroup per (sentence, frame) per iteration does the whole GL iteration for its frame:
//   overlap-add gather of the previous iteration's frames (<= 5 contributors per sample) with the
//   window-sum-square normalisation and the STFT's reflect padding -> window -> 2048-point real
//   FFT (1024-point complex Stockham radix-4 in LDS) -> X/|X| * S -> inverse real FFT -> window
//   -> store the frame.  Iterations ping-pong the frames buffer (a frame's neighbours still read
//   the previous iteration), one launch per iteration, replayed from a hipGraph.
// Roofline: HBM-bound by the algorithm's 6300 B per frame-iteration.
#include <cmath>
#include <map>
#include <tuple>
#include <vector>

#include "common.h"

using namespace tts;

namespace {

constexpr int NFFT = 2048;
constexpr int NB = 1025;  // bins
constexpr int NH = 1024;  // complex FFT size
constexpr int GL_THREADS = 256;

struct Geo {
    int hop, win, woff, winp;  // woff = (NFFT - win) / 2, winp = win rounded up to 4
};

struct GLConst {
    const float* win;   // [2048] padded periodic Hann
    const float* win2;  // [2048] win^2
    const float2* tw;   // [2048] e^{-2 pi i m / 2048}
};

__device__ __forceinline__ float2 cmul(float2 a, float2 b) { return float2{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ float2 cconj(float2 a) { return float2{a.x, -a.y}; }

// Stockham radix-4, 5 passes, 256 threads x 1 butterfly.  src -> result in dst (returned).
template <bool INV>
__device__ float2* fft1024(float2* src, float2* dst, const float2* __restrict__ tw) {
    const int j = threadIdx.x;
#pragma unroll
    for (int Ns = 1; Ns < NH; Ns *= 4) {
        const int k = j & (Ns - 1);
        float2 v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = src[j + r * 256];
        if (Ns > 1) {
#pragma unroll
            for (int r = 1; r < 4; ++r) {
                float2 w = tw[k * r * (512 / Ns)];
                if (INV) w = cconj(w);
                v[r] = cmul(v[r], w);
            }
        }
        const float2 a0 = float2{v[0].x + v[2].x, v[0].y + v[2].y};
        const float2 a1 = float2{v[0].x - v[2].x, v[0].y - v[2].y};
        const float2 a2 = float2{v[1].x + v[3].x, v[1].y + v[3].y};
        const float2 a3 = float2{v[1].x - v[3].x, v[1].y - v[3].y};
        // -i*a3 = (a3.y, -a3.x); +i*a3 = (-a3.y, a3.x)
        const float2 m3 = INV ? float2{-a3.y, a3.x} : float2{a3.y, -a3.x};
        const int idxD = (j / Ns) * Ns * 4 + k;
        dst[idxD] = float2{a0.x + a2.x, a0.y + a2.y};
        dst[idxD + Ns] = float2{a1.x + m3.x, a1.y + m3.y};
        dst[idxD + 2 * Ns] = float2{a0.x - a2.x, a0.y - a2.y};
        dst[idxD + 3 * Ns] = float2{a1.x - m3.x, a1.y - m3.y};
        __syncthreads();
        float2* t = src;
        src = dst;
        dst = t;
    }
    return src;
}

// Bijective XCD-aware remap: consecutive logical frames share an XCD (their OLA gathers
// re-read each other's frames through that XCD's L2).  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int n) {
    const int q = n >> 3, r = n & 7, x = bid & 7, i = bid >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// np.pad(..., mode='reflect') index map for a signal of length N (any overhang).
__device__ __forceinline__ int reflect_idx(int p, int N) {
    if (N == 1) return 0;
    const int period = 2 * (N - 1);
    int pp = p % period;
    if (pp < 0) pp += period;
    return pp < N ? pp : period - pp;
}

// y[p] of the previous iteration's iSTFT: overlap-add of the frames covering OLA position
// q = p + n_fft/2, divided by the window sum-square where it exceeds float32 tiny.
__device__ __forceinline__ float ola_sample(const float* __restrict__ fr, int q, int F, const Geo& g,
                                            const float* __restrict__ win2) {
    int ilo = q - g.woff - g.win + 1;
    ilo = ilo <= 0 ? 0 : (ilo + g.hop - 1) / g.hop;
    if (q < g.woff) return 0.f;
    int ihi = (q - g.woff) / g.hop;
    if (ihi > F - 1) ihi = F - 1;
    float y = 0.f, wss = 0.f;
    for (int i = ilo; i <= ihi; ++i) {
        const int o = q - i * g.hop;  // offset inside frame i (0..2047)
        y += fr[(int64_t)i * g.winp + (o - g.woff)];
        wss += win2[o];
    }
    return wss > 1.17549435e-38f ? y / wss : y;
}

// ---------------------------------------------------------------- |S|^power
struct MagArgs {
    int mode;  // TTS_GL_FROM_MEL / TTS_GL_FROM_LINEAR
    const float* spec;
    int n_in, Fmax;
    const int* F;
    const float* pinv;  // [1025][n_mels]
    float* S;
    float min_db, ref_db, power, max_norm;
    int signal_norm, symmetric, clip;
};

__device__ __forceinline__ float denorm_to_amp(float x, const MagArgs& a) {
    // _denormalize (utils/audio.py:96-112) then _db_to_amp(x + ref_level_db) (:125-126)
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
    return powf(10.f, (d + a.ref_db) * 0.05f);
}

__global__ __launch_bounds__(256) void gl_magnitude_kernel(const MagArgs a) {
    const int b = blockIdx.y;
    const int f0 = blockIdx.x * 16;
    const int Fb = a.F[b];
    if (f0 >= Fb) return;
    const int nf = min(16, Fb - f0);
    const float* sp = a.spec + ((int64_t)b * a.Fmax + f0) * a.n_in;
    float* S = a.S + ((int64_t)b * a.Fmax + f0) * NB;
    if (a.mode == TTS_GL_FROM_LINEAR) {
        for (int i = threadIdx.x; i < nf * NB; i += blockDim.x) S[i] = powf(denorm_to_amp(sp[i], a), a.power);
        return;
    }
    __shared__ float amp[16][80];
    for (int i = threadIdx.x; i < nf * a.n_in; i += blockDim.x) amp[i / a.n_in][i % a.n_in] = denorm_to_amp(sp[i], a);
    __syncthreads();
    // _mel_to_linear: max(1e-10, pinv(M) . S)  (utils/audio.py:64-66), then ** power
    for (int k = threadIdx.x; k < NB; k += blockDim.x) {
        const float* pr = a.pinv + (int64_t)k * a.n_in;
        float acc[16];
#pragma unroll
        for (int f = 0; f < 16; ++f) acc[f] = 0.f;
        for (int m = 0; m < a.n_in; ++m) {
            const float w = pr[m];
#pragma unroll
            for (int f = 0; f < 16; ++f) acc[f] += w * amp[f][m];
        }
        for (int f = 0; f < nf; ++f) S[(int64_t)f * NB + k] = powf(fmaxf(acc[f], 1e-10f), a.power);
    }
}

// ---------------------------------------------------------------- GL iteration
struct IterArgs {
    const float* S;       // [B][Fmax][1025]
    const float* prev;    // frames of the previous iteration (null for the initial iSTFT)
    float* next;          // frames written by this iteration
    const int* F;
    int Fmax;
    int B;
    Geo g;
    GLConst c;
    const double* phase_u;  // initial iSTFT only: [B][1025][Fmax] or null (device RNG)
    unsigned long long seed;
};

__device__ __forceinline__ double hash_uniform(unsigned long long seed, unsigned long long idx) {
    unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (idx + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

template <bool INIT>
__global__ __launch_bounds__(GL_THREADS) void gl_iter_kernel(const IterArgs a) {
    const int b = blockIdx.y;
    const int f = xcd_remap(blockIdx.x, gridDim.x);
    const int Fb = a.F[b];
    if (f >= Fb) return;
    const Geo g = a.g;
    const int tid = threadIdx.x;
    __shared__ __align__(16) float2 buf0[NH];
    __shared__ __align__(16) float2 buf1[NH];
    __shared__ __align__(16) float2 X[NB + 3];
    const float* Sf = a.S + ((int64_t)b * a.Fmax + f) * NB;

    if (!INIT) {
        // ---- STFT frame f of the previous iteration's signal (librosa stft, centre reflect pad)
        const int N = g.hop * (Fb - 1);
        const float* fr = a.prev + (int64_t)b * a.Fmax * g.winp;
        float* xr = reinterpret_cast<float*>(buf0);  // z[n] = x[2n] + i x[2n+1] == real x[0..2047]
        for (int n = tid; n < NFFT; n += GL_THREADS) {
            const float w = a.c.win[n];
            float v = 0.f;
            if (w != 0.f) {
                const int p = reflect_idx(f * g.hop + n - NFFT / 2, N);
                v = w * ola_sample(fr, p + NFFT / 2, Fb, g, a.c.win2);
            }
            xr[n] = v;
        }
        __syncthreads();
        float2* Z = fft1024<false>(buf0, buf1, a.c.tw);
        // real-FFT split + phase projection: X_k <- S_k * X_k / |X_k|   (angle(0) = 0 -> 1)
        for (int k = tid; k < NB; k += GL_THREADS) {
            const float2 zk = Z[k & (NH - 1)];
            const float2 zc = cconj(Z[(NH - k) & (NH - 1)]);
            const float2 E = float2{0.5f * (zk.x + zc.x), 0.5f * (zk.y + zc.y)};
            const float2 O = float2{0.5f * (zk.y - zc.y), -0.5f * (zk.x - zc.x)};  // -i (zk - zc) / 2
            const float2 Xk = float2{E.x + (a.c.tw[k].x * O.x - a.c.tw[k].y * O.y),
                                     E.y + (a.c.tw[k].x * O.y + a.c.tw[k].y * O.x)};
            const float r = sqrtf(Xk.x * Xk.x + Xk.y * Xk.y);
            const float s = Sf[k];
            X[k] = r > 0.f ? float2{s * (Xk.x / r), s * (Xk.y / r)} : float2{s, 0.f};
        }
    } else {
        // ---- initial phases exp(2 pi i U), U ~ U[0,1)  (utils/audio.py:183)
        for (int k = tid; k < NB; k += GL_THREADS) {
            const double u = a.phase_u ? a.phase_u[((int64_t)b * NB + k) * a.Fmax + f]
                                       : hash_uniform(a.seed, ((unsigned long long)b * NB + k) * 1048576ull + f);
            double sn, cs;
            sincos(2.0 * M_PI * u, &sn, &cs);
            const float s = Sf[k];
            X[k] = float2{(float)(s * cs), (float)(s * sn)};
        }
    }
    __syncthreads();
    // ---- inverse real FFT (istft: ifft of the Hermitian-extended spectrum, .real => Im X_0 = Im X_N/2 = 0)
    if (tid == 0) {
        X[0].y = 0.f;
        X[NB - 1].y = 0.f;
    }
    __syncthreads();
    for (int k = tid; k < NH; k += GL_THREADS) {
        const float2 xk = X[k];
        const float2 xc = cconj(X[NH - k]);
        const float2 E = float2{0.5f * (xk.x + xc.x), 0.5f * (xk.y + xc.y)};
        const float2 D = float2{0.5f * (xk.x - xc.x), 0.5f * (xk.y - xc.y)};
        const float2 w = cconj(a.c.tw[k]);
        const float2 O = cmul(D, w);
        buf0[k] = float2{E.x - O.y, E.y + O.x};  // E + i O
    }
    __syncthreads();
    const float2* z = fft1024<true>(buf0, buf1, a.c.tw);
    // ---- window and store the support [woff, woff+win)
    float* out = a.next + ((int64_t)b * a.Fmax + f) * g.winp;
    const float* zr = reinterpret_cast<const float*>(z);
    for (int n = tid; n < g.win; n += GL_THREADS) {
        const int m = g.woff + n;
        out[n] = a.c.win[m] * (zr[m] * (1.f / NH));
    }
}

// ---------------------------------------------------------------- final OLA + inverse pre-emphasis
struct FinArgs {
    const float* frames;
    const int* F;
    int Fmax, B;
    Geo g;
    GLConst c;
    float* y;  // [B][Nmax]
    int64_t Nmax;
};

__global__ void gl_ola_kernel(const FinArgs a) {
    const int b = blockIdx.y;
    const int Fb = a.F[b];
    const int N = a.g.hop * (Fb - 1);
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N) return;
    a.y[(int64_t)b * a.Nmax + p] = ola_sample(a.frames + (int64_t)b * a.Fmax * a.g.winp, p + NFFT / 2, Fb, a.g, a.c.win2);
}

// y[n] = x[n] + c*y[n-1] (scipy.signal.lfilter([1], [1, -c], x), utils/audio.py:133-136), fp64.
// One workgroup per sentence: chunked scan, carries combined serially in fixed order.
__global__ __launch_bounds__(1024) void preemph_scan_kernel(const float* y, int64_t Nmax, const int* F, int hop,
                                                            double coef, int apply, double* wav) {
    const int b = blockIdx.x;
    const int64_t N = (int64_t)hop * (F[b] - 1);
    const float* x = y + (int64_t)b * Nmax;
    double* o = wav + (int64_t)b * Nmax;
    const int T = blockDim.x, tid = threadIdx.x;
    const int64_t chunk = (N + T - 1) / T;
    const int64_t s0 = tid * chunk, s1 = s0 + chunk < N ? s0 + chunk : N;
    __shared__ double endv[1024];
    __shared__ double powc[1024];
    __shared__ double carry[1025];
    if (!apply) {
        for (int64_t i = tid; i < N; i += T) o[i] = (double)x[i];
        return;
    }
    double acc = 0.0, pc = 1.0;
    for (int64_t i = s0; i < s1; ++i) {
        acc = (double)x[i] + coef * acc;
        pc *= coef;
    }
    endv[tid] = acc;
    powc[tid] = pc;
    __syncthreads();
    if (tid == 0) {
        double c = 0.0;
        for (int i = 0; i < T; ++i) {
            carry[i] = c;
            c = endv[i] + powc[i] * c;
        }
    }
    __syncthreads();
    acc = carry[tid];
    for (int64_t i = s0; i < s1; ++i) {
        acc = (double)x[i] + coef * acc;
        o[i] = acc;
    }
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
    float *win = nullptr, *win2 = nullptr, *pinv = nullptr;
    float2* tw = nullptr;
    // workspace
    size_t S_floats = 0, fr_floats = 0, y_floats = 0;
    float *S = nullptr, *frames = nullptr, *y = nullptr;
    int* F = nullptr;
    int Fcap_B = 0;
    std::map<GraphKey, hipGraphExec_t> graphs;
    float last_ms = 0.f;
    int last_launches = 0;
    bool have_last = false;
    IterArgs last_iter{};
    FinArgs last_fin{};
    size_t last_fstride = 0;
};

extern "C" {

void tts_gl_destroy(tts_gl* g) {
    if (!g) return;
    if (g->stream) (void)hipStreamSynchronize(g->stream);
    for (auto& kv : g->graphs) (void)hipGraphExecDestroy(kv.second);
    for (void* p : {(void*)g->win, (void*)g->win2, (void*)g->pinv, (void*)g->tw, (void*)g->S, (void*)g->frames,
                    (void*)g->y, (void*)g->F})
        if (p) (void)hipFree(p);
    for (hipEvent_t e : {g->ev_in, g->ev_out, g->ev_t0, g->ev_t1})
        if (e) (void)hipEventDestroy(e);
    if (g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
}

tts_status tts_gl_create(const tts_audio_config* cfg, const float* inv_mel_basis, void* stream, tts_gl** out) {
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
    g->g.winp = (cfg->win_length + 3) / 4 * 4;
    hipStream_t s = static_cast<hipStream_t>(stream);
    // host tables in double, rounded once
    std::vector<float> win(NFFT, 0.f), win2(NFFT, 0.f);
    for (int n = 0; n < cfg->win_length; ++n) {
        const double w = 0.5 - 0.5 * std::cos(2.0 * M_PI * n / cfg->win_length);  // periodic Hann
        win[g->g.woff + n] = (float)w;
        win2[g->g.woff + n] = (float)(w * w);
    }
    std::vector<float2> tw(NFFT);
    for (int m = 0; m < NFFT; ++m)
        tw[m] = float2{(float)std::cos(2.0 * M_PI * m / NFFT), (float)-std::sin(2.0 * M_PI * m / NFFT)};
    auto fail = [&](hipError_t e, const char* what) {
        tts_status st = hip_fail(e, what, __FILE__, __LINE__);
        tts_gl_destroy(g);
        return st;
    };
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking)) != hipSuccess) return fail(e, "stream");
    if ((e = hipEventCreateWithFlags(&g->ev_in, hipEventDisableTiming)) != hipSuccess) return fail(e, "event");
    if ((e = hipEventCreateWithFlags(&g->ev_out, hipEventDisableTiming)) != hipSuccess) return fail(e, "event");
    if ((e = hipEventCreate(&g->ev_t0)) != hipSuccess) return fail(e, "event");
    if ((e = hipEventCreate(&g->ev_t1)) != hipSuccess) return fail(e, "event");
    if ((e = hipMalloc(&g->win, NFFT * 4)) != hipSuccess) return fail(e, "hipMalloc");
    if ((e = hipMalloc(&g->win2, NFFT * 4)) != hipSuccess) return fail(e, "hipMalloc");
    if ((e = hipMalloc(&g->tw, NFFT * sizeof(float2))) != hipSuccess) return fail(e, "hipMalloc");
    if ((e = hipMemcpy(g->win, win.data(), NFFT * 4, hipMemcpyHostToDevice)) != hipSuccess) return fail(e, "copy");
    if ((e = hipMemcpy(g->win2, win2.data(), NFFT * 4, hipMemcpyHostToDevice)) != hipSuccess) return fail(e, "copy");
    if ((e = hipMemcpy(g->tw, tw.data(), NFFT * sizeof(float2), hipMemcpyHostToDevice)) != hipSuccess)
        return fail(e, "copy");
    if (inv_mel_basis) {
        const size_t n = (size_t)NB * cfg->num_mels;
        if ((e = hipMalloc(&g->pinv, n * 4)) != hipSuccess) return fail(e, "hipMalloc");
        if ((e = hipMemcpy(g->pinv, inv_mel_basis, n * 4, hipMemcpyHostToDevice)) != hipSuccess) return fail(e, "copy");
    }
    (void)s;
    *out = g;
    return TTS_OK;
}

tts_status tts_gl_run(tts_gl* g, int mode, const float* spec, const int32_t* F, int B, int Fmax,
                      const double* phase_u, uint64_t seed, int iters, double* wav, void* stream) {
    TTS_CHECK(g && spec && F && wav && B >= 1 && Fmax >= 2 && iters >= 0, TTS_ERR_INVALID, "bad gl_run arguments");
    TTS_CHECK(mode == TTS_GL_FROM_MEL || mode == TTS_GL_FROM_LINEAR, TTS_ERR_INVALID, "bad mode");
    TTS_CHECK(mode == TTS_GL_FROM_LINEAR || g->pinv, TTS_ERR_INVALID, "mel mode needs inv_mel_basis at create");
    if (mode == TTS_GL_FROM_LINEAR)
        TTS_CHECK(g->cfg.power > 0, TTS_ERR_INVALID, "power must be > 0");
    for (int b = 0; b < B; ++b) TTS_CHECK(F[b] >= 2 && F[b] <= Fmax, TTS_ERR_INVALID, "F[b] out of range [2, Fmax]");
    hipStream_t cs = static_cast<hipStream_t>(stream);
    hipStream_t s = g->stream;
    const Geo geo = g->g;
    const int64_t Nmax = (int64_t)geo.hop * (Fmax - 1);
    // workspace (grow only; graphs keyed on shapes are invalidated when buffers move)
    const size_t needS = (size_t)B * Fmax * NB, needF = (size_t)2 * B * Fmax * geo.winp, needY = (size_t)B * Nmax;
    bool moved = false;
    auto grow = [&](float** p, size_t& have, size_t need) -> tts_status {
        if (need <= have) return TTS_OK;
        if (*p) TTS_HIP(hipFree(*p));
        *p = nullptr;
        TTS_HIP(hipMalloc(p, need * 4));
        have = need;
        moved = true;
        return TTS_OK;
    };
    TTS_HIP(hipStreamSynchronize(s));
    tts_status st;
    if ((st = grow(&g->S, g->S_floats, needS))) return st;
    if ((st = grow(&g->frames, g->fr_floats, needF))) return st;
    if ((st = grow(&g->y, g->y_floats, needY))) return st;
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
    TTS_HIP(hipEventRecord(g->ev_in, cs));
    TTS_HIP(hipStreamWaitEvent(s, g->ev_in, 0));
    TTS_HIP(hipMemcpyAsync(g->F, F, B * sizeof(int), hipMemcpyHostToDevice, s));
    MagArgs ma{};
    ma.mode = mode;
    ma.spec = spec;
    ma.n_in = mode == TTS_GL_FROM_MEL ? g->cfg.num_mels : NB;
    ma.Fmax = Fmax;
    ma.F = g->F;
    ma.pinv = g->pinv;
    ma.S = g->S;
    ma.min_db = g->cfg.min_level_db;
    ma.ref_db = g->cfg.ref_level_db;
    ma.power = g->cfg.power;
    ma.max_norm = g->cfg.max_norm;
    ma.signal_norm = g->cfg.signal_norm;
    ma.symmetric = g->cfg.symmetric_norm;
    ma.clip = g->cfg.clip_norm;
    hipLaunchKernelGGL(gl_magnitude_kernel, dim3((Fmax + 15) / 16, B), dim3(256), 0, s, ma);
    TTS_HIP(hipGetLastError());
    const size_t fstride = (size_t)B * Fmax * geo.winp;
    IterArgs ia{};
    ia.S = g->S;
    ia.F = g->F;
    ia.Fmax = Fmax;
    ia.B = B;
    ia.g = geo;
    ia.c = GLConst{g->win, g->win2, g->tw};
    ia.phase_u = phase_u;
    ia.seed = seed;
    ia.prev = nullptr;
    ia.next = g->frames;
    const dim3 grid(Fmax, B), block(GL_THREADS);
    hipLaunchKernelGGL(gl_iter_kernel<true>, grid, block, 0, s, ia);
    TTS_HIP(hipGetLastError());
    TTS_HIP(hipEventRecord(g->ev_t0, s));
    if (iters > 0) {
        GraphKey key{B, Fmax, iters};
        auto it = g->graphs.find(key);
        if (it == g->graphs.end()) {
            hipGraph_t graph = nullptr;
            TTS_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            for (int i = 0; i < iters; ++i) {
                IterArgs a = ia;
                a.phase_u = nullptr;
                a.prev = g->frames + (i & 1) * fstride;
                a.next = g->frames + ((i + 1) & 1) * fstride;
                hipLaunchKernelGGL(gl_iter_kernel<false>, grid, block, 0, s, a);
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
    TTS_HIP(hipEventRecord(g->ev_t1, s));
    FinArgs fa{};
    fa.frames = g->frames + (iters & 1) * fstride;
    fa.F = g->F;
    fa.Fmax = Fmax;
    fa.B = B;
    fa.g = geo;
    fa.c = ia.c;
    fa.y = g->y;
    fa.Nmax = Nmax;
    hipLaunchKernelGGL(gl_ola_kernel, dim3((Nmax + 255) / 256, B), dim3(256), 0, s, fa);
    TTS_HIP(hipGetLastError());
    hipLaunchKernelGGL(preemph_scan_kernel, dim3(B), dim3(1024), 0, s, g->y, Nmax, g->F, geo.hop,
                       g->cfg.preemphasis, g->cfg.preemphasis != 0.0 ? 1 : 0, wav);
    TTS_HIP(hipGetLastError());
    TTS_HIP(hipEventRecord(g->ev_out, s));
    TTS_HIP(hipStreamWaitEvent(cs, g->ev_out, 0));
    TTS_HIP(hipEventSynchronize(g->ev_t1));
    TTS_HIP(hipEventElapsedTime(&g->last_ms, g->ev_t0, g->ev_t1));
    g->last_launches = iters;
    g->have_last = true;
    g->last_iter = ia;
    g->last_fin = fa;
    g->last_fstride = fstride;
    return TTS_OK;
}

tts_status tts_gl_profile(tts_gl* g, int reps, float* kernel_ms, int n_kernels) {
    TTS_CHECK(g && kernel_ms && n_kernels >= TTS_GL_KERNELS && reps >= 1, TTS_ERR_INVALID, "bad profile arguments");
    TTS_CHECK(g->have_last, TTS_ERR_INVALID, "tts_gl_profile needs a previous tts_gl_run");
    hipStream_t s = g->stream;
    hipEvent_t ev[3];
    for (auto& e : ev) TTS_HIP(hipEventCreate(&e));
    const IterArgs& ia = g->last_iter;
    const dim3 grid(ia.Fmax, ia.B), block(GL_THREADS);
    double it_ms = 0.0, ola_ms = 0.0;
    for (int r = 0; r < reps; ++r) {
        IterArgs a = ia;
        a.phase_u = nullptr;
        a.prev = g->frames + (r & 1) * g->last_fstride;
        a.next = g->frames + ((r + 1) & 1) * g->last_fstride;
        TTS_HIP(hipEventRecord(ev[0], s));
        hipLaunchKernelGGL(gl_iter_kernel<false>, grid, block, 0, s, a);
        TTS_HIP(hipGetLastError());
        TTS_HIP(hipEventRecord(ev[1], s));
        FinArgs f = g->last_fin;
        f.frames = a.next;
        hipLaunchKernelGGL(gl_ola_kernel, dim3((f.Nmax + 255) / 256, f.B), dim3(256), 0, s, f);
        TTS_HIP(hipGetLastError());
        TTS_HIP(hipEventRecord(ev[2], s));
        TTS_HIP(hipEventSynchronize(ev[2]));
        float a_ms = 0.f, b_ms = 0.f;
        TTS_HIP(hipEventElapsedTime(&a_ms, ev[0], ev[1]));
        TTS_HIP(hipEventElapsedTime(&b_ms, ev[1], ev[2]));
        it_ms += a_ms;
        ola_ms += b_ms;
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    kernel_ms[0] = (float)(it_ms / reps);
    kernel_ms[1] = (float)(ola_ms / reps);
    return TTS_OK;
}

tts_status tts_gl_last_timing(tts_gl* g, float* loop_ms, int* launches) {
    TTS_CHECK(g && loop_ms && launches, TTS_ERR_INVALID, "null argument");
    *loop_ms = g->last_ms;
    *launches = g->last_launches;
    return TTS_OK;
}

}  // extern "C"

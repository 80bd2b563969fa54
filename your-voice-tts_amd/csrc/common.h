// Shared device/host helpers for libtts_hip (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/tts_hip.h"

namespace tts {

void set_error(const std::string& msg);
tts_status hip_fail(hipError_t e, const char* what, const char* file, int line);

#define TTS_HIP(call)                                                        \
    do {                                                                     \
        hipError_t _e = (call);                                              \
        if (_e != hipSuccess) return ::tts::hip_fail(_e, #call, __FILE__, __LINE__); \
    } while (0)

#define TTS_CHECK(cond, code, msg)           \
    do {                                             \
        if (!(cond)) {                               \
            ::tts::set_error(msg);                   \
            return code;                             \
        }                                            \
    } while (0)

// Pipeline mode (tts_synth_run, synth_api.hip; internal, not exported): while set, a stage runs its
// work on the caller's stream instead of its own (no event hand-off in or out), and leaves the
// completion checks that would block the host (encoder placement status, Griffin-Lim timing and
// status) pending for the pipeline to collect at its next synchronisation point.
void encoder_set_pipeline(tts_encoder* e, bool on);
// *placement_failed = 1: the resident encoder could not be placed, or one of its hand-off waits
// timed out: the caller reruns the encoder (with per-step launches)
tts_status encoder_pending_status(tts_encoder* e, int* placement_failed);
// the encoder handle's own ids / output buffers: a pipeline passes them as tts_encoder_run's ids /
// out to skip the staging copies (null ids buffer: B x Lmax exceeds the handle's capacity)
int32_t* encoder_ids_buffer(tts_encoder* e, int B, int Lmax);
float* encoder_out_buffer(tts_encoder* e);
void decoder_set_pipeline(tts_decoder* d, bool on);
// the decoder's mel history (sentence b at mel + b * sentence_floats, rows of nmel * r floats) and
// its device step counts, where a pipeline-mode run (decoder_set_pipeline) leaves its output
void decoder_histories(tts_decoder* d, const float** mel, int64_t* sentence_floats, const int** n_steps);
// work to enqueue behind the batch-1 resident launch before the host waits for it (null: none;
// cleared when pipeline mode ends); decoder_hook_ran: the last run enqueued it AND its result is the
// resident launch's (false after a multi-launch rerun: the caller enqueues that work again)
void decoder_set_post_hook(tts_decoder* d, void (*fn)(void*, hipStream_t), void* ctx);
bool decoder_hook_ran(tts_decoder* d);
// the next batch-1 resident runs read the sentence length from this device array (the encoder's own,
// encoder_lens_buffer) instead of uploading it, and one more status word is read back with the
// decoder's own (src -> pinned dst; the pipeline's deferred encoder status); clamp_dst (or null)
// receives the speculative Griffin-Lim frame counts (Readback below); cleared when pipeline mode ends
void decoder_set_pipeline_io(tts_decoder* d, const int* lens_dev, const int* rb_src, int* rb_dst, int* clamp_dst,
                             int clamp_max);
// the encoder's device length array, and its batch-1 resident status word with the pinned word the
// host reads it from; defer: a pipeline-mode batch-1 resident run leaves that read-back to the caller
const int* encoder_lens_buffer(tts_encoder* e);
void encoder_status_words(tts_encoder* e, const int** dev, int** host);
void encoder_set_defer_status(tts_encoder* e, bool defer);
// _add_speaker_embedding on an encoder output, on stream s (tts_encoder_add_speakers's body)
tts_status encoder_add_speakers(tts_encoder* e, float* enc, const int32_t* lens, const int32_t* speaker_ids, int B,
                                int Lmax, hipStream_t s);
// the next pipeline-mode run's lengths are already in encoder_lens_buffer (stage_ids): no upload
void encoder_set_lens_staged(tts_encoder* e, bool staged);
// postnet.hip: tts_postnet_run with device frame counts (T_dev[b] * tmul) and input rows mel_tmax
// frames apart (0 = Tmax); T holds the same counts on the host
tts_status postnet_run_dev(tts_postnet* p, const float* mel, int mel_tmax, const int* T_dev, int tmul, const int32_t* T,
                           int B, int Tmax, float* out, hipStream_t s);
void gl_set_pipeline(tts_gl* g, bool on);
// griffin_lim.hip: tts_gl_run with the frame counts also on the device (F_dev, or null); F_bound:
// F holds upper bounds only, F_dev (on the same stream) the counts
tts_status gl_run_dev(tts_gl* g, int mode, const float* spec, const int32_t* F, const int* F_dev, int B, int Fmax,
                      const double* phase_u, uint64_t seed, int iters, double* wav, hipStream_t stream,
                      bool F_bound = false);
tts_status gl_collect(tts_gl* g);  // waits for a pending run, sets its timing, checks its status
// whether gl_run_dev takes the persistent loop for this shape (host values only)
bool gl_persistent_path(tts_gl* g, int B, int Fmax, int frames_total, int iters);  // (caches per-F checks in g)
// phase_mt.hip: numpy's legacy np.random.rand(1025, F[b]) draws for b = 0..B-1 in order, continued
// on the device from the MT19937 state `state` ([dev] 624 key words + position, updated in place)
// into out [dev] fp64 [B][1025][Fmax] (F_dev on the device, read on stream s).  The stream is cut into
// chunks of MT_CHUNK_BLOCKS key blocks, each started by a GF(2) jump-ahead and generated by its own
// workgroup; `w` holds the caller's device workspace (grown on demand; the caller orders reuse).
constexpr int MT_MAX_BATCH = 1024;
struct MtWork {
    unsigned* xs = nullptr;             // the raw word stream, [blocks][624]
    size_t xs_words = 0;
    unsigned long long* polys = nullptr;  // jump polynomials of chunks 1.., [n][312]
    int npolys = 0;
    long long* meta = nullptr;          // position, draws, last block, sentence offsets
};
hipError_t mt_draw_phases(unsigned* state, const int* F_dev, int B, int Fmax, double* out, MtWork* w, hipStream_t s);
void mt_work_free(MtWork* w);
// wav_io.hip: Synthesizer.tts's join + save_wav's int16 conversion (tts_gl_save_pcm16's body)
hipError_t pcm16_join(const double* wav, int64_t pitch, const int64_t* start_dev, int64_t total, int B, int gap,
                      double peak, unsigned long long* peak_bits, int16_t* out, hipStream_t s);

// Persistent kernels (in-launch hand-offs between workgroups: resident decoder / encoder, persistent
// Griffin-Lim) are only correct if every workgroup of the grid is resident at once.  This checks
// the grid against the device's occupancy (the kernel's workgroups per CU x CUs, the CU count
// optionally capped by the TTS_CU_CAP environment variable, which tests use to force the fallback)
// and, if it fits, launches `fn` with a PLAIN hipLaunchKernel by default: the check does not
// guarantee co-residency when other work occupies CUs, so correctness rests on the kernels' bounded
// waits plus their status word (the decoder / encoder then rerun multi-launch, the persistent
// Griffin-Lim raises with a NaN waveform).  TTS_COOP=1 uses hipLaunchCooperativeKernel instead
// (≈30 µs more per launch).  *launched = false (and hipSuccess) when the grid cannot fit: nothing
// ran and the caller takes its multi-launch path.
hipError_t launch_persistent(const void* fn, dim3 grid, dim3 block, void** args, size_t smem, hipStream_t s,
                             bool* launched);
// rows [B][K] (row stride ld) -> their fragment-order mirror (frag_idx, ntf m-tiles)
hipError_t frag_mirror(const float* src, int64_t ld, int B, int K, float* dst, int ntf, hipStream_t s);
// the CU count launch_persistent plans with (device CUs, capped by TTS_CU_CAP)
int usable_cus();
// record `ev` on `s` and wait for it by polling (runtime.hip: the blocking wait's wake-up latency
// sits on the synthesis critical path)
hipError_t spin_sync(hipStream_t s, hipEvent_t ev);
hipError_t spin_wait(hipEvent_t ev);  // the same wait on an event already recorded
// Small device -> pinned-host read-back in ONE launch (runtime.hip: readback_kernel) instead of one
// copy launch per array: up to 4 int arrays (system-scope stores, visible to the host once an
// event recorded after the launch has completed), plus an optional clamp of frame counts for a
// Griffin-Lim enqueued before they are known: clamp_dst[b] = src[b] if 2 <= src[b] <= clamp_max,
// else 0 (every launch of that run exits at once; the caller redoes the sentence).
struct Readback {
    const int* src[4];
    int n[4];
    int* dst[4];
    int count;
    const int* clamp_src;
    int* clamp_dst;
    int clamp_n, clamp_max;
    int* seq_dst;  // pinned coherent host word written `seq` after every other word (release), or null
    int seq;
};
hipError_t readback(const Readback& r, hipStream_t s);
// Host wait for a pinned coherent word that a kernel on `s` sets to `want` with a system-scope release
// (Readback::seq_dst, the Griffin-Lim overlap-add's status sequence): polled for up to TTS_SPIN_MS,
// then the stream is synchronised.  Replaces an event record + query: each event marker in a stream
// was measured to hold the GPU ~5.8 us between the kernels around it (round-4 kernel trace).
hipError_t spin_word(const int* p, int want, hipStream_t s);
// the device side of spin_word: thread 0 of the launch, after every thread's earlier stores
__device__ __forceinline__ void release_word_system(int* p, int v) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// A batch-1 sentence's ids (and its length) written to device arrays by one kernel whose argument
// block carries them (runtime.hip), in place of two host-to-device copies: on this runtime a small
// pageable-or-pinned H2D copy was measured to hold the host until its stream drained (~50 µs of
// idle device at every pipelined sentence boundary).
constexpr int STAGE_IDS_MAX = 512;
struct StageIds {
    int32_t* ids;
    int* lens;
    int n, len;  // ids to write, the length value
    int32_t v[STAGE_IDS_MAX];
};
hipError_t stage_ids(const StageIds& a, hipStream_t s);

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int WAVE = 64;

// v_mfma_f32_16x16x4_f32: lane l supplies A[l&15][l>>4] and B[l>>4][l&15];
// D lane l holds C[(l>>4)*4 + r][l&15], r = 0..3.  Exact f32 fma chain.
// Fragment-order mirror of an activation matrix [rows][K] (rows padded to nt m-tiles of 16, K a
// multiple of 16): element (b, k) sits where lane (b & 15) + 16 ((k & 15) >> 2), component k & 3
// of the v_mfma_f32_16x16x4_f32 A-operand float4 of (chunk k >> 4, m-tile b >> 4) loads it, so a
// wave's operand load is one contiguous 1 KiB instead of 16 rows x 64 B (sgemm.h).
__device__ __forceinline__ int64_t frag_idx(int b, int k, int nt) {
    return ((((int64_t)(k >> 4) * nt + (b >> 4)) * 64 + (b & 15) + 16 * ((k & 15) >> 2)) << 2) + (k & 3);
}

__device__ __forceinline__ floatx4 mfma16x16x4(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
// DPP wave reductions (VALU data-parallel-primitive lanes moves: no LDS round trip per level as
// __shfl_xor's ds_bpermute has).  Inclusive row scans by row_shr 1/2/4/8, then row_bcast:15 and
// row_bcast:31 carry rows into lane 63; the total is read from lane 63 (wave-uniform result).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_move(float v, float identity) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(identity), __float_as_int(v), CTRL, ROW_MASK,
                                                      0xf, false));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
    v += dpp_move<0x111, 0xf>(v, 0.f);  // row_shr:1
    v += dpp_move<0x112, 0xf>(v, 0.f);  // row_shr:2
    v += dpp_move<0x114, 0xf>(v, 0.f);  // row_shr:4
    v += dpp_move<0x118, 0xf>(v, 0.f);  // row_shr:8
    v += dpp_move<0x142, 0xa>(v, 0.f);  // row_bcast:15 into rows 1, 3
    v += dpp_move<0x143, 0xc>(v, 0.f);  // row_bcast:31 into rows 2, 3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
    const float id = -INFINITY;
    v = fmaxf(v, dpp_move<0x111, 0xf>(v, id));
    v = fmaxf(v, dpp_move<0x112, 0xf>(v, id));
    v = fmaxf(v, dpp_move<0x114, 0xf>(v, id));
    v = fmaxf(v, dpp_move<0x118, 0xf>(v, id));
    v = fmaxf(v, dpp_move<0x142, 0xa>(v, id));
    v = fmaxf(v, dpp_move<0x143, 0xc>(v, id));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// (value, index) max with first-index tie break (torch.argmax / max(dim) semantics).
__device__ __forceinline__ void wave_argmax(float& v, int& i) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        float ov = __shfl_xor(v, o, 64);
        int oi = __shfl_xor(i, o, 64);
        if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
    }
}

// Block reductions; `scratch` must hold >= 2*nwaves entries; all threads get the result.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) scratch[w] = v;
    __syncthreads();
    float s = 0.f;
    for (int k = 0; k < nw; ++k) s += scratch[k];  // fixed order: deterministic
    return s;
}
__device__ __forceinline__ float block_max(float v, float* scratch) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_max(v);
    __syncthreads();
    if (lane == 0) scratch[w] = v;
    __syncthreads();
    float s = scratch[0];
    for (int k = 1; k < nw; ++k) s = fmaxf(s, scratch[k]);
    return s;
}
__device__ __forceinline__ int block_argmax(float v, int i, float* scratch, int* iscratch) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    wave_argmax(v, i);
    __syncthreads();
    if (lane == 0) { scratch[w] = v; iscratch[w] = i; }
    __syncthreads();
    float bv = scratch[0];
    int bi = iscratch[0];
    for (int k = 1; k < nw; ++k)
        if (scratch[k] > bv || (scratch[k] == bv && iscratch[k] < bi)) { bv = scratch[k]; bi = iscratch[k]; }
    return bi;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// Recurrent-cell gate nonlinearities (the resident decoders' and encoder's LSTM / GRU cells, on
// every step's critical path) from the hardware exp2 / reciprocal instead of the libm sequences
// (~27 and ~40 dependent instructions; round 5: -0.17 us/step on the resident Tacotron2 step):
// sigmoid within ~3 ulp; tanh within ~5e-7 relative, an odd Taylor polynomial below |x| = 0.5
// (no cancellation near 0) and 1 - 2 / (1 + e^2|x|) above.
__device__ __forceinline__ float sigmoid_cell(float x) {
    return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-x * 1.4426950408889634f));
}
__device__ __forceinline__ float tanh_cell(float x) {
    const float ax = fabsf(x);
    const float big = 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(ax * 2.8853900817779268f));
    const float x2 = x * x;
    float p = -1.45583438705e-3f;  // tanh x = x (1 - x^2/3 + 2x^4/15 - ... ), terms through x^15
    p = fmaf(p, x2, 3.59212803657e-3f);
    p = fmaf(p, x2, -8.86323552990e-3f);
    p = fmaf(p, x2, 2.18694885362e-2f);
    p = fmaf(p, x2, -5.39682539683e-2f);
    p = fmaf(p, x2, 1.33333333333e-1f);
    p = fmaf(p, x2, -3.33333333333e-1f);
    p = fmaf(p, x2, 1.f);
    return ax < 0.5f ? x * p : copysignf(big, x);
}
// tanh from the hardware exp2 / reciprocal (2 transcendental issues instead of the libm
// range-reduction sequence): absolute error <= ~3e-7 over the whole range, saturating exactly
// to +-1.  Used where tanh feeds a weighted sum (attention energies), not a recurrence.
__device__ __forceinline__ float tanh_fast(float x) {
    const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);  // exp(2x)
    return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
}

}  // namespace tts

// Whole-sentence synthesis in one call: ids -> encoder -> decoder -> postnet -> Griffin-Lim, the
// chain utils/synthesis.py:synthesis runs (model.inference, :50-57 -> ap.inv_mel_spectrogram of the
// postnet output, :69-77) for Tacotron2 without speaker embedding.  Every stage is the same entry
// point the host package binds one by one (same numerics, bitwise); this call only removes the
// host round trips between them: one H2D of the ids, the decoder's stop-step readback (the
// sentence length is decided on the device) and the stages' own completion waits.  The stages
// run in pipeline mode (common.h) and the call returns once Griffin-Lim is enqueued: the
// waveform is ready when the caller's stream reaches it.  Above 512 frames Griffin-Lim runs on a
// second stream of this handle, so call k+1's encoder + decoder (which read only host inputs and
// this handle's buffers) need not wait for call k's Griffin-Lim; the stage buffers Griffin-Lim
// reads (mel_post, its compacted copy) alternate per call.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"

struct tts_synth {
    tts_encoder* e = nullptr;
    tts_decoder* d = nullptr;
    tts_postnet* p = nullptr;
    tts_gl* g = nullptr;
    int r = 1, nmel = 80, hop = 0;
    int32_t* ids = nullptr;  // [dev] [B][Lmax]
    float *enc = nullptr, *mel = nullptr, *stop = nullptr;
    // Griffin-Lim inputs, one pair per call parity: call k+1's postnet writes the other pair while
    // call k's Griffin-Lim reads this one (call k+2 comes after call k+1 collected call k's run)
    float *post[2] = {nullptr, nullptr}, *spec[2] = {nullptr, nullptr};
    size_t ids_n = 0, enc_n = 0, mel_n = 0, stop_n = 0, spec_n = 0;
    std::vector<int32_t> steps;
    // encoder -> decoder -> postnet on `stream`, Griffin-Lim on `gl_stream` (default priorities: see
    // tts_synth_create).  Neither front stage touches caller
    // memory, so `stream` does not wait for the caller's; Griffin-Lim waits for the caller's
    // stream (it writes the caller's waveform buffer) and for the postnet, and the caller's stream
    // waits for Griffin-Lim.
    hipStream_t stream = nullptr, gl_stream = nullptr;
    hipEvent_t ev_in = nullptr, ev_post = nullptr, ev_out = nullptr;
    // pinned host staging of ids / lens / frames, alternated per call: call k reuses call k-2's
    // buffer, whose copies completed before call k-1's decoder synchronisation and Griffin-Lim
    // collection
    int32_t* pin[2] = {nullptr, nullptr};
    size_t pin_n[2] = {0, 0};
    unsigned calls = 0;
    int* fspec = nullptr;  // [dev] frame count of a speculative batch-1 Griffin-Lim (synth_stages)
    // the caller's stream the last batch-1 run worked on (synth_stages), or null: tts_synth_sync waits
    // for it (that run's stages, down to the de-emphasis writing the waveform, are on it only)
    hipStream_t last_cs = nullptr;
};

namespace {
template <typename T>
tts_status grow(T** p, size_t& have, size_t need) {
    if (need <= have) return TTS_OK;
    if (*p) TTS_HIP(hipFree(*p));
    *p = nullptr;
    TTS_HIP(hipMalloc(reinterpret_cast<void**>(p), need * sizeof(T)));
    have = need;
    return TTS_OK;
}

// stages run in pipeline mode (common.h) for the duration of one tts_synth_run
struct PipelineScope {
    tts_synth* s;
    explicit PipelineScope(tts_synth* x) : s(x) { set(true); }
    ~PipelineScope() { set(false); }
    void set(bool on) {
        tts::encoder_set_pipeline(s->e, on);
        tts::decoder_set_pipeline(s->d, on);
        tts::gl_set_pipeline(s->g, on);
    }
};

// the stages of one tts_synth_run after the host staging (defined below)
tts_status synth_stages(tts_synth* s, int32_t* h_ids, int32_t* h_lens, const int32_t* spk, int32_t* h_frames, int B,
                        int Lmax, int max_steps, int gl_iters, uint64_t seed, double* wav, int64_t wav_cap,
                        int32_t* frames, void* stream);
tts_status synth_run(tts_synth* s, const int32_t* ids, const int32_t* lens, const int32_t* spk, int B, int Lmax,
                     int max_steps, int gl_iters, uint64_t seed, double* wav, int64_t wav_cap, int32_t* frames,
                     void* stream);
}  // namespace

extern "C" {

tts_status tts_synth_create(tts_encoder* e, tts_decoder* d, tts_postnet* p, tts_gl* g, int r, int n_mel, int hop,
                            tts_synth** out) {
    TTS_CHECK(e && d && p && g && out, TTS_ERR_INVALID, "null handle");
    TTS_CHECK(r >= 1 && n_mel >= 1 && hop >= 1, TTS_ERR_INVALID, "bad r / n_mel / hop");
    tts_synth* s = new tts_synth;
    s->e = e;
    s->d = d;
    s->p = p;
    s->g = g;
    s->r = r;
    s->nmel = n_mel;
    s->hop = hop;
    // both streams at the default priority: with a high-priority front stream (round 3) every few
    // launches after the resident decoder waited ~35 us for its waves to be dispatched (postnet
    // layers, the Griffin-Lim magnitude / initial iSTFT / overlap-add / de-emphasis launches:
    // +0.2 ms per configs[1] sentence; rocprofv3 SQ counters showed the same busy cycles at 3x the
    // wall time).  TTS_STREAM_PRIO=1 restores the priorities (measurement only).
    int prio_lo = 0, prio_hi = 0;
    if (const char* v = getenv("TTS_STREAM_PRIO"); v && v[0] == '1')
        if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_lo = prio_hi = 0;
    if (hipStreamCreateWithPriority(&s->stream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
        hipStreamCreateWithPriority(&s->gl_stream, hipStreamNonBlocking, prio_lo) != hipSuccess ||
        hipEventCreateWithFlags(&s->ev_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&s->ev_post, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&s->ev_out, hipEventDisableTiming) != hipSuccess ||
        hipMalloc(&s->fspec, 4 * sizeof(int)) != hipSuccess) {
        tts_synth_destroy(s);
        tts::set_error("tts_synth_create: stream / event creation failed");
        return TTS_ERR_HIP;
    }
    *out = s;
    return TTS_OK;
}

void tts_synth_destroy(tts_synth* s) {
    if (!s) return;
    for (hipStream_t q : {s->stream, s->gl_stream})
        if (q) (void)hipStreamSynchronize(q);
    // a batch-1 run worked on the caller's stream, which may be gone by now: wait for the device
    if (s->last_cs) (void)hipDeviceSynchronize();
    if (tts::gl_collect(s->g) != TTS_OK)  // the last pipelined run's status was never collected
        std::fprintf(stderr, "tts_synth_destroy: the last run failed: %s\n", tts_last_error());
    for (void* q : {(void*)s->ids, (void*)s->enc, (void*)s->mel, (void*)s->stop, (void*)s->post[0],
                    (void*)s->post[1], (void*)s->spec[0], (void*)s->spec[1], (void*)s->fspec})
        if (q) (void)hipFree(q);
    for (int32_t* q : s->pin)
        if (q) (void)hipHostFree(q);
    for (hipEvent_t ev : {s->ev_in, s->ev_post, s->ev_out})
        if (ev) (void)hipEventDestroy(ev);
    for (hipStream_t q : {s->stream, s->gl_stream})
        if (q) (void)hipStreamDestroy(q);
    delete s;
}

tts_status tts_synth_run(tts_synth* s, const int32_t* ids, const int32_t* lens, int B, int Lmax, int max_steps,
                         int gl_iters, uint64_t seed, double* wav, int64_t wav_cap, int32_t* frames, void* stream) {
    return synth_run(s, ids, lens, nullptr, B, Lmax, max_steps, gl_iters, seed, wav, wav_cap, frames, stream);
}

tts_status tts_synth_run_speakers(tts_synth* s, const int32_t* ids, const int32_t* lens, const int32_t* speaker_ids,
                                  int B, int Lmax, int max_steps, int gl_iters, uint64_t seed, double* wav,
                                  int64_t wav_cap, int32_t* frames, void* stream) {
    TTS_CHECK(speaker_ids, TTS_ERR_INVALID, "null speaker_ids");
    return synth_run(s, ids, lens, speaker_ids, B, Lmax, max_steps, gl_iters, seed, wav, wav_cap, frames, stream);
}
}  // extern "C"

namespace {
tts_status synth_run(tts_synth* s, const int32_t* ids, const int32_t* lens, const int32_t* spk, int B, int Lmax,
                     int max_steps, int gl_iters, uint64_t seed, double* wav, int64_t wav_cap, int32_t* frames,
                     void* stream) {
    TTS_CHECK(s && ids && lens && wav && frames && B >= 1 && Lmax >= 2 && max_steps >= 1 && gl_iters >= 0,
              TTS_ERR_INVALID, "bad synth arguments");
    hipStream_t ss = s->stream;
    const int cap = max_steps + 21;  // decoder steps_cap (>= max_steps + 20)
    const size_t T = (size_t)cap * s->r;
    tts_status st;
    hipStream_t cs = static_cast<hipStream_t>(stream);
    // buffers are only (re)allocated with nothing of this pipeline in flight (a batch-1 run works on
    // the caller's stream: synth_stages)
    const bool regrow = (size_t)B * Lmax > s->ids_n || (size_t)B * Lmax * 512 > s->enc_n ||
                        (size_t)B * T * s->nmel > s->mel_n || (size_t)B * cap > s->stop_n;
    const int par = s->calls & 1;
    const size_t pin_need = (size_t)B * Lmax + 2 * (size_t)B;
    if (regrow || pin_need > s->pin_n[par]) {
        TTS_HIP(hipStreamSynchronize(ss));
        TTS_HIP(hipStreamSynchronize(s->gl_stream));
        TTS_HIP(hipStreamSynchronize(cs));
    }
    if ((st = grow(&s->ids, s->ids_n, (size_t)B * Lmax))) return st;
    if ((st = grow(&s->enc, s->enc_n, (size_t)B * Lmax * 512))) return st;
    if ((st = grow(&s->mel, s->mel_n, (size_t)B * T * s->nmel))) return st;
    if ((st = grow(&s->stop, s->stop_n, (size_t)B * cap))) return st;
    if (!s->post[0] || s->spec_n < s->mel_n) {
        // mel_post and the compacted GL input share the mel buffer's capacity (mel_n only grows
        // on a regrow, which drained both streams above)
        for (int k = 0; k < 2; ++k) {
            if (s->post[k]) TTS_HIP(hipFree(s->post[k]));
            if (s->spec[k]) TTS_HIP(hipFree(s->spec[k]));
            s->post[k] = s->spec[k] = nullptr;
        }
        for (int k = 0; k < 2; ++k) {
            TTS_HIP(hipMalloc(&s->post[k], s->mel_n * sizeof(float)));
            TTS_HIP(hipMalloc(&s->spec[k], s->mel_n * sizeof(float)));
        }
        s->spec_n = s->mel_n;
    }
    if (pin_need > s->pin_n[par]) {
        if (s->pin[par]) TTS_HIP(hipHostFree(s->pin[par]));
        s->pin[par] = nullptr;
        TTS_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->pin[par]), pin_need * sizeof(int32_t)));
        s->pin_n[par] = pin_need;
    }
    int32_t* h_ids = s->pin[par];
    int32_t* h_lens = h_ids + (size_t)B * Lmax;
    int32_t* h_frames = h_lens + B;
    std::copy(ids, ids + (size_t)B * Lmax, h_ids);
    std::copy(lens, lens + B, h_lens);
    // a call that fails after staging may still have copies from pin[par] in flight: drain them
    // before returning, so the next call can restage the same buffer
    st = synth_stages(s, h_ids, h_lens, spk, h_frames, B, Lmax, max_steps, gl_iters, seed, wav, wav_cap, frames, stream);
    if (st) {
        (void)hipStreamSynchronize(s->stream);
        (void)hipStreamSynchronize(s->gl_stream);
        (void)hipStreamSynchronize(cs);
        return st;
    }
    ++s->calls;  // only now: a failed call leaves the parity (and its drained buffers) to the next
    return TTS_OK;
}
}  // namespace

extern "C" {
tts_status tts_synth_sync(tts_synth* s) {
    TTS_CHECK(s, TTS_ERR_INVALID, "null handle");
    TTS_HIP(hipStreamSynchronize(s->stream));
    TTS_HIP(hipStreamSynchronize(s->gl_stream));
    // a batch-1 run's stages ran on the caller's stream (no event marks their end: ADVICE r5)
    if (s->last_cs) TTS_HIP(hipStreamSynchronize(s->last_cs));
    return tts::gl_collect(s->g);
}

}  // extern "C"

namespace {
tts_status synth_stages(tts_synth* s, int32_t* h_ids, int32_t* h_lens, const int32_t* spk, int32_t* h_frames, int B,
                        int Lmax, int max_steps, int gl_iters, uint64_t seed, double* wav, int64_t wav_cap,
                        int32_t* frames, void* stream) {
    hipStream_t cs = static_cast<hipStream_t>(stream);
    // a batch-1 run (the latency path) works on the caller's stream itself: every stage in stream
    // order behind the caller's earlier work, and no cross-stream event between this call's stages
    // or against the next call (each record / wait held the GPU ~6 us: the first Griffin-Lim
    // launch waited on the caller's stream, the next call's first launch on the previous call's
    // end-of-run event).  TTS_SYNTH_OWN_STREAM=1 restores the handle's own stream.
    static const bool own_stream = [] {
        const char* v = getenv("TTS_SYNTH_OWN_STREAM");
        return v && v[0] == '1';
    }();
    hipStream_t ss = B == 1 && !own_stream ? cs : s->stream;
    s->last_cs = ss == cs ? cs : nullptr;
    const int cap = max_steps + 21;
    const size_t T = (size_t)cap * s->r;
    tts_status st;
    const int par = s->calls & 1;
    PipelineScope scope(s);
    // batch > 1: the front stages do not wait for the caller's stream (they read host inputs and
    // write this handle's buffers only), nor for the previous call's Griffin-Lim (batch 1 runs on
    // the caller's stream, in its order).  The persistent Griffin-Lim
    // (whose workgroups wait on each other) only runs on this same stream (<= 512 frames, below),
    // so it never shares the device with this call's resident launches.  A cross-stream Griffin-Lim
    // is the non-persistent per-iteration form; if its workgroups keep a resident encoder /
    // decoder workgroup from being placed, that launch's bounded waits drain it and the stage
    // re-runs multi-launch (decoder_api.hip, encoder_api.hip): slower, never wrong.
    // the ids go straight into the encoder's own buffer, and the decoder reads the encoder's own
    // output buffer (no device-to-device staging copies)
    int32_t* ids_dev = tts::encoder_ids_buffer(s->e, B, Lmax);
    if (!ids_dev) ids_dev = s->ids;
    float* const enc = tts::encoder_out_buffer(s->e);
    if (B == 1 && Lmax <= tts::STAGE_IDS_MAX && ids_dev != s->ids) {
        // batch 1: ids and length through one kernel's arguments (common.h: stage_ids)
        tts::StageIds sa;
        sa.ids = ids_dev;
        sa.lens = const_cast<int*>(tts::encoder_lens_buffer(s->e));
        sa.n = Lmax;
        sa.len = h_lens[0];
        std::copy(h_ids, h_ids + Lmax, sa.v);
        TTS_HIP(tts::stage_ids(sa, ss));
        tts::encoder_set_lens_staged(s->e, true);
    } else {
        TTS_HIP(hipMemcpyAsync(ids_dev, h_ids, sizeof(int32_t) * (size_t)B * Lmax, hipMemcpyHostToDevice, ss));
        tts::encoder_set_lens_staged(s->e, false);
    }
    s->steps.assign(B, 0);
    // batch 1: the postnet is enqueued behind the resident decoder launch before the host waits for
    // it (device step counts; tiles sized for Tp = min(T, 1024) frames, the tiles past the sentence
    // exit), so the device goes from the decoder to the postnet without waiting for the host to wake
    // up.  Tp bounds the frames that run gives (the small-batch conv kernel's limit, independent of
    // the step cap): a longer sentence is redone after the wait, like the speculative Griffin-Lim.
    const float* hist = nullptr;
    int64_t sent_floats = 0;
    const int* n_dev = nullptr;
    tts::decoder_histories(s->d, &hist, &sent_floats, &n_dev);
    float* const post = s->post[par];
    // ... and, when its frame count can only take the persistent Griffin-Lim (<= 256 frames, r = 1),
    // Griffin-Lim too: sized for Ts = min(256, T) frames, reading the count the decoder's read-back
    // launch clamps into fspec (a longer sentence makes it an empty run, redone below)
    const int Ts = (int)std::min<size_t>(256, T);
    const int Tp = (int)std::min<size_t>(1024, T);
    static const bool no_spec = [] {  // measurement only: no speculative Griffin-Lim in the hook
        const char* v = getenv("TTS_NO_SPEC_GL");
        return v && v[0] == '1';
    }();
    const bool spec_gl = B == 1 && s->r == 1 && !no_spec && wav_cap >= (int64_t)s->hop * (Ts - 1) &&
                         tts::gl_persistent_path(s->g, 1, Ts, Ts, gl_iters);
    struct Hook {
        tts_synth* s;
        const float* hist;
        int mel_tmax;
        const int* n_dev;
        float* post;
        int T, Tp;
        tts_status st;
        bool spec_gl;
        int Ts;
        uint64_t seed;
        int iters;
        double* wav;
        hipStream_t cs;
        bool gl_done;
    } hook{s, hist, (int)(sent_floats / s->nmel), n_dev, post, (int)T, Tp, TTS_OK, spec_gl, Ts, seed, gl_iters, wav, cs, false};
    auto hook_fn = [](void* c, hipStream_t q) {
        Hook* h = static_cast<Hook*>(c);
        const int32_t Tcap[1] = {h->Tp};
        h->st = tts::postnet_run_dev(h->s->p, h->hist, h->mel_tmax, h->n_dev, h->s->r, Tcap, 1, h->T, h->post, q);
        if (h->st || !h->spec_gl) return;
        // Griffin-Lim writes the caller's waveform: after the caller's stream (the same stream: in
        // order already).  An idle caller stream needs no cross-stream wait (its marker would hold
        // the GPU ~5.8 us before the first Griffin-Lim launch)
        const hipError_t idle = q == h->cs ? hipSuccess : hipStreamQuery(h->cs);
        if (idle != hipSuccess && idle != hipErrorNotReady) {
            h->st = TTS_ERR_HIP;
            tts::set_error("tts_synth_run: caller stream query failed");
            return;
        }
        if (idle == hipErrorNotReady &&
            (hipEventRecord(h->s->ev_in, h->cs) != hipSuccess || hipStreamWaitEvent(q, h->s->ev_in, 0) != hipSuccess)) {
            h->st = TTS_ERR_HIP;
            tts::set_error("tts_synth_run: event hand-off failed");
            return;
        }
        const int32_t Fb[1] = {h->Ts};
        h->st = tts::gl_run_dev(h->s->g, TTS_GL_FROM_MEL, h->post, Fb, h->s->fspec, 1, h->Ts, nullptr, h->seed, h->iters,
                                h->wav, q, true);
        h->gl_done = h->st == TTS_OK;
    };
    // batch 1: the sentence length from the encoder's device copy, the encoder's status word read back
    // with the decoder's (one launch), the speculative Griffin-Lim's frame count clamped by it
    if (B == 1) {
        const int* est = nullptr;
        int* ehost = nullptr;
        tts::encoder_status_words(s->e, &est, &ehost);
        tts::encoder_set_defer_status(s->e, est != nullptr);
        tts::decoder_set_pipeline_io(s->d, tts::encoder_lens_buffer(s->e), est, ehost, spec_gl ? s->fspec : nullptr, Ts);
    }
    static const bool no_hook = [] {  // measurement only: postnet and Griffin-Lim after the host's wait
        const char* v = getenv("TTS_NO_HOOK");
        return v && v[0] == '1';
    }();
    tts::decoder_set_post_hook(s->d, B == 1 && !no_hook ? +hook_fn : nullptr, &hook);
    for (int attempt = 0;; ++attempt) {
        if ((st = tts_encoder_run(s->e, ids_dev, h_lens, B, Lmax, enc, ss))) return st;
        // Tacotron2._add_speaker_embedding (models/tacotron2.py:65, 91-100)
        if (spk && (st = tts::encoder_add_speakers(s->e, enc, h_lens, spk, B, Lmax, ss))) return st;
        // synchronises ss: the encoder's placement status is then readable
        st = tts_decoder_run(s->d, enc, h_lens, B, Lmax, max_steps, cap, s->mel, s->stop, nullptr, s->steps.data(), ss);
        if (!st) st = hook.st;
        if (st) {
            tts::decoder_set_post_hook(s->d, nullptr, nullptr);
            return st;
        }
        int rerun = 0;
        if ((st = tts::encoder_pending_status(s->e, &rerun))) return st;
        if (!rerun) break;
        TTS_CHECK(attempt == 0, TTS_ERR_HIP, "encoder rerun failed (internal error)");
    }
    int Fmax = 0;
    for (int b = 0; b < B; ++b) {
        h_frames[b] = s->steps[b] * s->r;
        Fmax = std::max(Fmax, (int)h_frames[b]);
    }
    TTS_CHECK(Fmax >= 2, TTS_ERR_INVALID, "a sentence decoded to fewer than 2 frames");
    TTS_CHECK(wav_cap >= (int64_t)B * s->hop * (Fmax - 1), TTS_ERR_INVALID, "wav buffer too small");
    std::copy(h_frames, h_frames + B, frames);
    const bool post_done = tts::decoder_hook_ran(s->d) && Fmax <= Tp;
    const bool gl_done = post_done && hook.gl_done && Fmax <= Ts;
    tts::decoder_set_post_hook(s->d, nullptr, nullptr);
    if (!post_done) {
        // the postnet reads the decoder's mel history in place, with the step counts the decoder left
        // on the device (pipeline mode: no history copies, no frame-count upload)
        if ((st = tts::postnet_run_dev(s->p, hist, (int)(sent_floats / s->nmel), n_dev, s->r, h_frames, B, (int)T, post, ss)))
            return st;
    }
    const float* spec = post;
    if (B > 1) {  // GL input is [B][Fmax][nmel]: compact the rows of each sentence
        const size_t row = (size_t)s->nmel * sizeof(float);
        TTS_HIP(hipMemcpy2DAsync(s->spec[par], Fmax * row, post, T * row, Fmax * row, B, hipMemcpyDeviceToDevice, ss));
        spec = s->spec[par];
    }
    // Small jobs (<= 512 frames: the persistent Griffin-Lim, whose spinning grid must not share the
    // device with the next call's resident launches anyway) stay on the front stream: no
    // cross-queue hand-offs on the latency-bound batch-1 path.  Larger ones move to gl_stream,
    // so the next call's encoder + decoder need not wait for them.
    int frames_total = 0;
    for (int b = 0; b < B; ++b) frames_total += h_frames[b];
    const bool same = frames_total <= 512;
    hipStream_t gs = same ? ss : s->gl_stream;
    if (gl_done) {  // enqueued behind the decoder already (hook_fn)
        if (ss != cs) {
            TTS_HIP(hipEventRecord(s->ev_out, ss));
            TTS_HIP(hipStreamWaitEvent(cs, s->ev_out, 0));
        }
        return TTS_OK;
    }
    if (gs != cs) TTS_HIP(hipEventRecord(s->ev_in, cs));
    if (!same) {
        TTS_HIP(hipEventRecord(s->ev_post, ss));
        TTS_HIP(hipStreamWaitEvent(gs, s->ev_post, 0));
    }
    if (gs != cs) TTS_HIP(hipStreamWaitEvent(gs, s->ev_in, 0));
    // shorter sentences leave their waveform tail unwritten: zero it
    if (B > 1) TTS_HIP(hipMemsetAsync(wav, 0, sizeof(double) * (size_t)B * s->hop * (Fmax - 1), gs));
    // at r = 1 the decoder's device step counts are the frame counts: no upload
    if ((st = tts::gl_run_dev(s->g, TTS_GL_FROM_MEL, spec, h_frames, s->r == 1 ? n_dev : nullptr, B, Fmax, nullptr, seed,
                              gl_iters, wav, gs)))
        return st;
    if (gs != cs) {
        TTS_HIP(hipEventRecord(s->ev_out, gs));
        TTS_HIP(hipStreamWaitEvent(cs, s->ev_out, 0));
    }
    return TTS_OK;
}
}  // namespace

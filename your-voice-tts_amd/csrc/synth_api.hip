// Whole-sentence synthesis in one call: ids -> encoder -> decoder -> postnet -> Griffin-Lim, the
// chain utils/synthesis.py:synthesis runs (model.inference, :50-57 -> ap.inv_mel_spectrogram of the
// postnet output, :69-77) for Tacotron2 without speaker embedding.  Every stage is the same entry
// point the host package binds one by one (same numerics, bitwise); this call only removes the
// host round trips between them: one H2D of the ids, the decoder's stop-step readback (the
// sentence length is decided on the device) and the stages' own completion waits.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "common.h"

struct tts_synth {
    tts_encoder* e = nullptr;
    tts_decoder* d = nullptr;
    tts_postnet* p = nullptr;
    tts_gl* g = nullptr;
    int r = 1, nmel = 80, hop = 0;
    int32_t* ids = nullptr;  // [dev] [B][Lmax]
    float *enc = nullptr, *mel = nullptr, *stop = nullptr, *post = nullptr, *spec = nullptr;
    size_t ids_n = 0, enc_n = 0, mel_n = 0, stop_n = 0, spec_n = 0;
    std::vector<int32_t> steps;
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
    *out = s;
    return TTS_OK;
}

void tts_synth_destroy(tts_synth* s) {
    if (!s) return;
    for (void* q : {(void*)s->ids, (void*)s->enc, (void*)s->mel, (void*)s->stop, (void*)s->post, (void*)s->spec})
        if (q) (void)hipFree(q);
    delete s;
}

tts_status tts_synth_run(tts_synth* s, const int32_t* ids, const int32_t* lens, int B, int Lmax, int max_steps,
                         int gl_iters, uint64_t seed, double* wav, int64_t wav_cap, int32_t* frames, void* stream) {
    TTS_CHECK(s && ids && lens && wav && frames && B >= 1 && Lmax >= 2 && max_steps >= 1 && gl_iters >= 0,
              TTS_ERR_INVALID, "bad synth arguments");
    hipStream_t cs = static_cast<hipStream_t>(stream);
    const int cap = max_steps + 21;  // decoder steps_cap (>= max_steps + 20)
    const size_t T = (size_t)cap * s->r;
    tts_status st;
    if ((st = grow(&s->ids, s->ids_n, (size_t)B * Lmax))) return st;
    if ((st = grow(&s->enc, s->enc_n, (size_t)B * Lmax * 512))) return st;
    if ((st = grow(&s->mel, s->mel_n, (size_t)B * T * s->nmel))) return st;
    if ((st = grow(&s->stop, s->stop_n, (size_t)B * cap))) return st;
    if (!s->post || s->spec_n < s->mel_n) {
        // mel_post and the compacted GL input share the mel buffer's capacity
        if (s->post) TTS_HIP(hipFree(s->post));
        if (s->spec) TTS_HIP(hipFree(s->spec));
        s->post = s->spec = nullptr;
        TTS_HIP(hipMalloc(&s->post, s->mel_n * sizeof(float)));
        TTS_HIP(hipMalloc(&s->spec, s->mel_n * sizeof(float)));
        s->spec_n = s->mel_n;
    }
    TTS_HIP(hipMemcpyAsync(s->ids, ids, sizeof(int32_t) * (size_t)B * Lmax, hipMemcpyHostToDevice, cs));
    if ((st = tts_encoder_run(s->e, s->ids, lens, B, Lmax, s->enc, cs))) return st;
    s->steps.assign(B, 0);
    if ((st = tts_decoder_run(s->d, s->enc, lens, B, Lmax, max_steps, cap, s->mel, s->stop, nullptr, s->steps.data(),
                              cs)))
        return st;
    int Fmax = 0;
    for (int b = 0; b < B; ++b) {
        frames[b] = s->steps[b] * s->r;
        Fmax = std::max(Fmax, (int)frames[b]);
    }
    TTS_CHECK(Fmax >= 2, TTS_ERR_INVALID, "a sentence decoded to fewer than 2 frames");
    TTS_CHECK(wav_cap >= (int64_t)B * s->hop * (Fmax - 1), TTS_ERR_INVALID, "wav buffer too small");
    if ((st = tts_postnet_run(s->p, s->mel, frames, B, (int)T, s->post, cs))) return st;
    const float* spec = s->post;
    if (B > 1) {  // GL input is [B][Fmax][nmel]: compact the rows of each sentence; shorter
                  // sentences leave their waveform tail unwritten: zero it
        const size_t row = (size_t)s->nmel * sizeof(float);
        TTS_HIP(hipMemcpy2DAsync(s->spec, Fmax * row, s->post, T * row, Fmax * row, B, hipMemcpyDeviceToDevice, cs));
        spec = s->spec;
        TTS_HIP(hipMemsetAsync(wav, 0, sizeof(double) * (size_t)B * s->hop * (Fmax - 1), cs));
    }
    return tts_gl_run(s->g, TTS_GL_FROM_MEL, spec, frames, B, Fmax, nullptr, seed, gl_iters, wav, cs);
}

}  // extern "C"

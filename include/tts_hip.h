/*
 * tts_hip.h — C-ABI of libtts_hip.so, the MI355X (gfx950) synthesis path of the
 * prototypefund/your-voice-TTS drop-in.
 *
 * The reference has no FFI for this path: it is pure Python on stock PyTorch ops and librosa
 * (SURVEY.md §0.1).  Each entry point below replaces one reference call site; the host package
 * (your-voice-tts_amd/) binds them with ctypes and keeps the reference's Python signatures.
 *
 * Conventions
 *   - Plain pointers and sizes only.  Pointers marked [dev] are device (HBM) pointers, [host]
 *     are host pointers.  `stream` is a hipStream_t passed as void* (NULL = default stream).
 *   - Caller owns all input/output buffers; the library owns weights, workspace and graphs.
 *   - Every call returns a tts_status; tts_last_error() gives the message of the last failure
 *     on the calling thread.  No exceptions cross the ABI.
 *   - A handle is not reentrant: one thread/stream per handle at a time (the reference decoder
 *     keeps per-call state on the module and is not reentrant either, layers/tacotron2.py:161-177).
 *   - Model arithmetic is fp32 (as the reference's torch modules); Griffin-Lim magnitudes, FFTs
 *     and the inverse pre-emphasis are fp64 (scipy.fftpack / scipy.signal.lfilter precision).
 */
#ifndef TTS_HIP_H
#define TTS_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int tts_status;
#define TTS_OK 0
#define TTS_ERR_INVALID 1     /* bad argument / shape / missing weight            */
#define TTS_ERR_HIP 2         /* HIP runtime error (message in tts_last_error)    */
#define TTS_ERR_UNSUPPORTED 3 /* configuration the path does not implement        */
#define TTS_ERR_NOMEM 4

typedef struct tts_encoder tts_encoder;
typedef struct tts_decoder tts_decoder;
typedef struct tts_postnet tts_postnet;
typedef struct tts_gl tts_gl;
typedef struct tts_tacotron tts_tacotron;

/* One weight tensor in the reference's own state_dict layout (fp32, contiguous, [dev]). */
typedef struct tts_tensor {
    const char* key;   /* reference state_dict key, e.g. "decoder.attention_rnn.weight_ih" */
    const float* data; /* [dev] fp32                                                        */
    int64_t numel;
} tts_tensor;

/* Replaces the embedding lookup + Encoder.inference of Tacotron2.inference (models/tacotron2.py:
 * 63-64, layers/tacotron2.py:48-83): 3 x (Conv1d k=5 + BatchNorm + ReLU) and the bidirectional
 * LSTM.  `tensors` must hold embedding.weight and every encoder.* key. */
tts_status tts_encoder_create(const tts_tensor* tensors, int n_tensors, int max_batch, int max_len,
                              void* stream, tts_encoder** out);
void tts_encoder_destroy(tts_encoder* e);
/*   ids  [dev]  int32 [B][Lmax] character ids (entries past lens[b] ignored)
 *   lens [host] int32 [B], 1 <= lens[b] <= Lmax
 *   out  [dev]  fp32 [B][Lmax][512]; each sentence is encoded at its own length, rows past
 *                lens[b] are zero. */
tts_status tts_encoder_run(tts_encoder* e, const int32_t* ids, const int32_t* lens, int B, int Lmax,
                           float* out, void* stream);
/* Same with the BiLSTM state carried (Encoder.inference_truncated, layers/tacotron2.py:85-93):
 *   state_in  [dev] fp32 [4][B][256] = (h_fwd, h_bwd, c_fwd, c_bwd) initial state, or NULL (zeros)
 *   state_out [dev] fp32 [4][B][256] final state (h_n, c_n per direction), or NULL. */
tts_status tts_encoder_run_state(tts_encoder* e, const int32_t* ids, const int32_t* lens, int B, int Lmax,
                                 const float* state_in, float* state_out, float* out, void* stream);

/* Tacotron2._add_speaker_embedding (models/tacotron2.py:65, 91-100) on an encoder output:
 * enc[b][t] += speaker_embedding.weight[speaker_ids[b]] for t < lens[b] (rows past stay zero).
 * The handle must have been created with speaker_embedding.weight among its tensors.
 *   enc [dev] fp32 [B][Lmax][512]; lens, speaker_ids [host] int32 [B] (B <= 64) */
tts_status tts_encoder_add_speakers(tts_encoder* e, float* enc, const int32_t* lens, const int32_t* speaker_ids, int B,
                                    int Lmax, void* stream);

/* 1 if the last run's BiLSTM took the resident (one co-resident launch) path, 0 for the per-step
 * launches (batches, or a device where the resident grid cannot be co-resident). */
tts_status tts_encoder_last_path(tts_encoder* e, int* resident);

/* Decoder flags: the arguments of layers/tacotron2.py:98-100 (Decoder.__init__) that change
 * inference numerics, as mapped from the JSON config by utils/generic_utils.py:275-288. */
typedef struct tts_decoder_config {
    int r;                 /* frames per step (config "r")                                 */
    int attn_norm;         /* 0 = softmax, 1 = sigmoid (common_layers.py:239-245)          */
    int forward_attn;      /* use_forward_attn                                             */
    int trans_agent;       /* transition_agent                                             */
    int forward_attn_mask; /* forward_attn_mask (synthesize.py:86 forces 1)                */
    int location_attn;     /* location_attn                                                */
    int windowing;         /* windowing (attn_win), eval-only window (common_layers.py:184) */
    int max_batch;         /* workspace capacity: sentences per call (<= 64)              */
    int max_len;           /* workspace capacity: encoder length L (<= 1024)              */
    int max_steps;         /* workspace capacity: decoder steps (max_decoder_steps)        */
} tts_decoder_config;

/* Replaces the construction + load_state_dict of layers/tacotron2.py:97-150 (Decoder).
 * `tensors` must hold every decoder.* key of the reference state_dict for this config; they
 * are repacked into the library's MFMA-fragment layout (the caller may free them after).
 * prenet_type "bn" (common_layers.py:28-70) is selected by the presence of the
 * decoder.prenet.layers.{0,1}.bn.* keys (eval-mode BatchNorm1d, folded into the prenet at create;
 * tts_tacotron_create does the same for its decoder prenet). */
tts_status tts_decoder_create(const tts_decoder_config* cfg, const tts_tensor* tensors, int n_tensors,
                              void* stream, tts_decoder** out);
void tts_decoder_destroy(tts_decoder* d);

/* Replaces Decoder.inference (layers/tacotron2.py:249-285) for a padded batch of sentences,
 * with per-sentence semantics identical to the reference run alone at batch 1:
 *   enc      [dev]  fp32 [B][Lmax][512] encoder outputs (rows >= lens[b] ignored)
 *   lens     [host] int32 [B] encoder lengths L_b (2 <= L_b <= Lmax <= cfg.max_len)
 *   max_steps        the reference's max_decoder_steps (<= cfg.max_steps)
 *   mel      [dev]  fp32 [B][steps_cap*r][80]  mel frames (decoder_output, time-major)
 *   stop     [dev]  fp32 [B][steps_cap]        sigmoid(stop token)
 *   align    [dev]  fp32 [B][steps_cap][Lmax]  attention weights per step (may be NULL)
 *   n_steps  [host] int32 [B] out: decoder steps taken by each sentence
 * steps_cap must be >= max_steps + 20 (the reference can run up to 20 steps past the cap once
 * every stop flag is set, layers/tacotron2.py:271-277).  Entries past n_steps[b] are left
 * untouched.  Synchronises `stream` once per chunk of steps to read the stop flags. */
tts_status tts_decoder_run(tts_decoder* d, const float* enc, const int32_t* lens, int B, int Lmax,
                           int max_steps, int steps_cap, float* mel, float* stop, float* align,
                           int32_t* n_steps, void* stream);

/* Continuous mode: replaces Decoder.inference_truncated (layers/tacotron2.py:287-328).  Same
 * arguments as tts_decoder_run, batch 1 only; the attention-LSTM / decoder-LSTM states, the
 * context and the memory (last mel frame) carry over from the previous batch-1 run on this handle,
 * the attention and stop-rule state restart. */
tts_status tts_decoder_run_continue(tts_decoder* d, const float* enc, const int32_t* lens, int B, int Lmax,
                                    int max_steps, int steps_cap, float* mel, float* stop, float* align,
                                    int32_t* n_steps, void* stream);

/* Teacher forcing: replaces Decoder.forward(inputs, memories, mask) (layers/tacotron2.py:227-247)
 * in eval mode.  Step t decodes from the go frame (t = 0) or teacher row t-1 (80*r values: frames
 * (t-1)r .. tr-1), with no stop rule: exactly `steps` steps for every sentence, each sentence at its
 * own encoder length (padding positions are never attended, as the reference's mask would do).
 *   memories [dev] fp32 [B][mem_ldb] teacher frames, row t at t * 80 * r
 *   mel   [dev] fp32 [B][steps][80*r]; stop [dev] fp32 [B][steps] stopnet LOGITS (no sigmoid, as
 *         Decoder.forward returns them); align [dev] fp32 [B][steps][Lmax] or null. */
tts_status tts_decoder_run_teacher(tts_decoder* d, const float* enc, const int32_t* lens, int B, int Lmax,
                                   const float* memories, int64_t mem_ldb, int steps, float* mel, float* stop,
                                   float* align, void* stream);

/* Per-step timing of the last tts_decoder_run (ms of GPU time of the step loop, steps run). */
tts_status tts_decoder_last_timing(tts_decoder* d, float* loop_ms, int* steps_run);

/* Which implementation ran the last tts_decoder_run / _continue (no reference counterpart):
 * *resident = 1 for the resident single-launch batch-1 decoder (every step weight held on chip
 * by 256 workgroups, hand-offs in device memory), 2 for the resident batch decoder (the same for
 * up to 4 sentences per launch, both LSTMs' rows in registers; consecutive launches for larger
 * batches), 0 for the per-step multi-launch hipGraph path.  The batch-1 path serves L <= 256 under
 * every Tacotron2 attention configuration, the batch path 2 <= B with every L_b <= 256 under those
 * without location features, windowing or transition agent; both need >= 256 compute units.
 * TTS_RESIDENT=0 / TTS_RESIDENT_BATCH=0 in the environment at tts_decoder_create disable them. */
tts_status tts_decoder_last_path(tts_decoder* d, int* resident);
/* The requests the resident decoder serves on this handle now: batches of at most *max_batch
 * sentences of encoder length <= *max_len (both 0: the handle runs multi-launch only, e.g. after
 * repeated placement failures).  Callers that split a request (Synthesizer.tts's dispatch) gate on it. */
tts_status tts_decoder_resident_limits(tts_decoder* d, int* max_batch, int* max_len);

/* Measurement only: re-runs the last resident batch-1 sentence with phase timers and returns the
 * mean microseconds per decoder step of each phase, us[0..15] on compute unit 0 and us[16..31] on
 * the attention compute unit (n >= 32): 0 attention-LSTM early part + wait pre1, 1 prenet-2 row
 * (0-1 on the prenet compute units), 2 wait prenet-2, 3 attention-LSTM prenet part, 4 cell + gather
 * h_att, 5 query row + decoder-LSTM early part, 6 wait query, 7 energies + max(alpha), 8 weights,
 * context, publish, 9 next-step prefetch (6-9 attention CU only), 10 wait context, 11 decoder-LSTM
 * context part, 12 cell + gather h_dec, 13 fused mel / prenet-1 / stop rows (wave 2); 14 and 15 split
 * 7 and 8 (candidate energies up to their barrier; window weights + context before publishing). */
#define TTS_RESIDENT_PHASES 16
tts_status tts_decoder_resident_phases(tts_decoder* d, float* us, int n);
// Measurement only: re-runs the last resident sentence with per-CU event stamps (no phase marks) and
// returns n >= 256*64*12 wall-clock ticks [CU][step < 64][event]: P1, B1, h_att published, B3, B4,
// h_dec published, B6, pre1 row published, query row published, and on the attention CUs A1 (query
// gathered), A2 (candidate energies), context published (0 = not reached).
tts_status tts_decoder_resident_trace(tts_decoder* d, long long* ticks, int64_t n);

/* Measurement only (no reference counterpart): re-runs up to `reps` steps of the last
 * tts_decoder_run's batch eagerly, with a HIP event before/after every kernel on the stream it
 * is launched on, and returns the mean duration (ms) of each step kernel, in launch order:
 * prenet2, attention-LSTM, query, attention, decoder-LSTM, fused mel/prenet1/stop.
 * Leaves the decoder state mid-sentence (the next tts_decoder_run re-initialises it). */
#define TTS_DECODER_STEP_KERNELS 6
tts_status tts_decoder_profile(tts_decoder* d, int reps, float* kernel_ms, int n_kernels);

/* Replaces Postnet (layers/tacotron2.py:30-45) + the residual add of models/tacotron2.py:69-70:
 * out = mel + postnet(mel), per sentence at its own length (zero padding past T_b).
 * `tensors` must hold the postnet.* keys. */
tts_status tts_postnet_create(const tts_tensor* tensors, int n_tensors, int n_mel, void* stream,
                              tts_postnet** out);
void tts_postnet_destroy(tts_postnet* p);
/*   mel [dev] fp32 [B][Tmax][n_mel] time-major; T [host] int32 [B]; out [dev] same shape. */
tts_status tts_postnet_run(tts_postnet* p, const float* mel, const int32_t* T, int B, int Tmax,
                           float* out, void* stream);

/* Audio parameters of AudioProcessor (utils/audio.py:12-54, 114-119). */
typedef struct tts_audio_config {
    int n_fft;          /* (num_freq-1)*2, must be 2048 */
    int hop_length;     /* frame_shift_ms * sample_rate / 1000 */
    int win_length;     /* frame_length_ms * sample_rate / 1000, <= n_fft */
    int num_mels;
    float min_level_db, ref_level_db, power, max_norm;
    double preemphasis; /* lfilter coefficient, kept in double as the reference's Python float */
    int signal_norm, symmetric_norm, clip_norm;
} tts_audio_config;

#define TTS_GL_FROM_MEL 0     /* AudioProcessor.inv_mel_spectrogram (utils/audio.py:164-172) */
#define TTS_GL_FROM_LINEAR 1  /* AudioProcessor.inv_spectrogram     (utils/audio.py:154-162) */

/* inv_mel_basis: [host] fp64 [n_fft/2+1][num_mels] = pinv(mel basis) (utils/audio.py:64-66);
 * may be NULL when only the linear path is used.  Magnitudes, FFTs and the phase are float64,
 * the STFT is rounded to complex64 and the signal kept float32, as librosa 0.6.2 does. */
tts_status tts_gl_create(const tts_audio_config* cfg, const double* inv_mel_basis, void* stream, tts_gl** out);
void tts_gl_destroy(tts_gl* g);

/* Batched Griffin-Lim vocoder: replaces inv_mel_spectrogram / inv_spectrogram, i.e.
 * denormalise -> dB->amp -> [pinv mel->linear] -> ^power -> _griffin_lim (utils/audio.py:182-201,
 * librosa 0.6.2 stft/istft) -> inverse pre-emphasis (lfilter, utils/audio.py:133-136).
 *   spec    [dev]  fp32 [B][Fmax][n_in] frame-major (n_in = num_mels or n_fft/2+1 by mode)
 *   F       [host] int32 [B] frames per sentence (>= 2)
 *   phase_u [dev]  fp64 [B][n_fft/2+1][Fmax] initial phases as U[0,1) draws (the reference's
 *                  np.random.rand(*S.shape)), or NULL: drawn on device from `seed`
 *   wav     [dev]  fp64 [B][hop*(Fmax-1)]: sentence b fills its first hop*(F_b-1) samples */
tts_status tts_gl_run(tts_gl* g, int mode, const float* spec, const int32_t* F, int B, int Fmax,
                      const double* phase_u, uint64_t seed, int iters, double* wav, void* stream);

/* numpy-stream initial phases.  The reference draws each sentence's initial Griffin-Lim phases
 * with np.random.rand(*S.shape) from numpy's global legacy generator (utils/audio.py:183), sentence
 * after sentence (server/synthesizer.py:145-158).  tts_gl_set_phase_state takes that generator's
 * state (np.random.get_state(): MT19937 key[624] and position 0..624) and arms the handle: every
 * following tts_gl_run with phase_u == NULL (and the runs of a tts_synth on this handle) draws its
 * phases from it ON THE DEVICE, one [n_fft/2+1][F_b] draw per sentence in batch order, bitwise the
 * values np.random.rand returns, and advances the state; key == NULL disarms (device-seeded phases
 * again).  tts_gl_get_phase_state waits for the last draw and returns the state numpy would hold
 * after the same draws (np.random.set_state it back).  tts_gl_draw_phases draws into phase_u [dev]
 * fp64 [B][n_fft/2+1][Fmax] directly (F [host] int32 [B], 0 <= F[b] <= Fmax, B <= 1024). */
tts_status tts_gl_set_phase_state(tts_gl* g, const uint32_t* key, int pos);
tts_status tts_gl_get_phase_state(tts_gl* g, uint32_t* key, int* pos);
tts_status tts_gl_draw_phases(tts_gl* g, const int32_t* F, int B, int Fmax, double* phase_u, void* stream);

/* Synthesizer.tts's join + AudioProcessor.save_wav's int16 conversion (server/synthesizer.py:157-161,
 * utils/audio.py:56-58), on the device: sentence b's first n[b] samples, each sentence followed by
 * `gap` zeros (10000 in the reference), scaled by 32767 / max(0.01, peak) and truncated to int16, with
 * numpy's float64 arithmetic (the bytes of the reference's wav).  peak < 0: max |y| over the request;
 * peak >= 0: that value (a sharded request's all-ranks maximum).
 *   wav [dev] fp64 [B][pitch]; n [host] int64 [B]; out [dev] int16 [sum(n[b] + gap)] */
tts_status tts_gl_save_pcm16(tts_gl* g, const double* wav, int64_t pitch, const int64_t* n, int B, int gap,
                             double peak, int16_t* out, void* stream);

/* Mel analysis for GST style wavs: AudioProcessor.melspectrogram (utils/audio.py:146-152) as used by
 * compute_style_mel (utils/synthesis.py:28-35): pre-emphasis FIR, librosa 0.6.2 stft (float64 FFT,
 * complex64 result), |D|, mel projection (float64), amp->dB, _normalize.
 *   mel_basis [host] fp64 [num_mels][n_fft/2+1] (librosa filters.mel), set once per handle
 *   wav [dev] fp64 [B][Nmax]; N [host] int32 [B] (>= 2); mel [dev] fp32 [B][Fmax][num_mels]
 *   (frame-major; sentence b has 1 + N[b]/hop frames, the rest zero). */
tts_status tts_gl_set_mel_basis(tts_gl* g, const double* mel_basis);
tts_status tts_gl_melspectrogram(tts_gl* g, const double* wav, const int32_t* N, int B, int64_t Nmax, float* mel,
                                 int Fmax, void* stream);

/* Time of the last tts_gl_run's iteration loop (ms, GPU) and kernel launches in it. */
tts_status tts_gl_last_timing(tts_gl* g, float* loop_ms, int* launches);

/* Iteration loop the last tts_gl_run took: TTS_GL_PATH_UNFUSED (overlap-add launch + per-frame
 * STFT/iSTFT launch per iteration), TTS_GL_PATH_FUSED (one launch per iteration), or
 * TTS_GL_PATH_PERSISTENT (every iteration in one co-resident launch, up to 512 frames in all: one
 * workgroup per frame, one per compute unit up to 256 workgroups and two per compute unit above;
 * when the grid cannot be co-resident the run falls back to the fused loop, bitwise the same
 * waveform). */
#define TTS_GL_PATH_UNFUSED 0
#define TTS_GL_PATH_FUSED 1
#define TTS_GL_PATH_PERSISTENT 2
tts_status tts_gl_last_path(tts_gl* g, int* path);

/* Measurement only: re-runs `reps` GL iterations of the last tts_gl_run's batch eagerly with
 * HIP events around each kernel on its stream; returns mean ms of [per-frame STFT/iSTFT kernel,
 * overlap-add kernel] (one iteration launches both).  Clobbers the internal frame and signal
 * buffers (not the caller's outputs). */
#define TTS_GL_KERNELS 2
tts_status tts_gl_profile(tts_gl* g, int reps, float* kernel_ms, int n_kernels);

/* ---------------------------------------------------------------- whole-sentence synthesis
 * Replaces utils/synthesis.py:synthesis for Tacotron2 (model.inference, :50-57,
 * then ap.inv_mel_spectrogram of the postnet output, :69-77) in ONE call over the handles above:
 * tts_encoder_run -> tts_decoder_run -> tts_postnet_run -> tts_gl_run (mel mode, device phases
 * from `seed`), bitwise the same as calling them one by one, without the host round trips in
 * between.  The handles stay owned by the caller and must outlive the tts_synth. */
typedef struct tts_synth tts_synth;
tts_status tts_synth_create(tts_encoder* e, tts_decoder* d, tts_postnet* p, tts_gl* g, int r, int n_mel, int hop,
                            tts_synth** out);
void tts_synth_destroy(tts_synth* s);
/*   ids    [host] int32 [B][Lmax]; lens [host] int32 [B], 2 <= lens[b] <= Lmax
 *   wav    [dev]  fp64 [B][hop*(Fmax-1)] out, Fmax = max frames[b] (wav_cap = elements available)
 *   frames [host] int32 [B] out: mel frames of each sentence (decoder steps * r); sentence b's
 *          waveform is the first hop*(frames[b]-1) samples of its row, the rest zero. */
tts_status tts_synth_run(tts_synth* s, const int32_t* ids, const int32_t* lens, int B, int Lmax, int max_steps,
                         int gl_iters, uint64_t seed, double* wav, int64_t wav_cap, int32_t* frames, void* stream);
/* tts_synth_run for a multi-speaker Tacotron2 (utils/synthesis.py:synthesis with speaker_id):
 * the speaker embedding is added to the encoder output (tts_encoder_add_speakers) before the decoder.
 *   speaker_ids [host] int32 [B] */
tts_status tts_synth_run_speakers(tts_synth* s, const int32_t* ids, const int32_t* lens, const int32_t* speaker_ids,
                                  int B, int Lmax, int max_steps, int gl_iters, uint64_t seed, double* wav,
                                  int64_t wav_cap, int32_t* frames, void* stream);
/* tts_synth_run returns once Griffin-Lim is enqueued; its completion status (a persistent loop's
 * hand-off timeout) is otherwise collected by the next run.  This waits for the last run and
 * returns that status.  A failed run's waveform is NaN, never a plausible-looking signal. */
tts_status tts_synth_sync(tts_synth* s);

/* ---------------------------------------------------------------- Tacotron / TacotronGST
 * SURVEY config 5 (config_tacotron_gst.json) and config_tacotron.json: the r-frames-per-step
 * Tacotron family, models/tacotron.py / models/tacotrongst.py. */
typedef struct tts_tacotron_config {
    int r;                 /* frames per step                                                  */
    int memory_size;       /* decoder memory queue (<= 0 means r); only memory_size == r       */
    int attn_norm;         /* 0 = softmax, 1 = sigmoid                                         */
    int forward_attn, trans_agent, forward_attn_mask, location_attn, windowing;
    int gst;               /* 1: TacotronGST (gst.* weights present), 0: Tacotron              */
    int num_speakers;      /* > 1: speaker_embedding.weight present                            */
    int max_batch;         /* workspace capacity: sentences per call (<= 64)                   */
    int max_len;           /* workspace capacity: encoder length (<= 1024, 512 with location)  */
    int max_steps;         /* workspace capacity: decoder steps (max_decoder_steps)            */
} tts_tacotron_config;

/* Replaces construction + load_state_dict of TacotronGST / Tacotron (models/tacotrongst.py:10-45,
 * models/tacotron.py:9-43).  `tensors` hold the model's state_dict entries (fp32 [dev]). */
tts_status tts_tacotron_create(const tts_tacotron_config* cfg, const tts_tensor* tensors, int n_tensors,
                               void* stream, tts_tacotron** out);
void tts_tacotron_destroy(tts_tacotron* t);

/* Replaces the embedding + Encoder (Prenet + CBHG, layers/tacotron.py:209-243) +
 * _add_speaker_embedding + GST add of TacotronGST.inference (models/tacotrongst.py:65-73):
 *   ids         [dev]  int32 [B][Lmax]
 *   lens        [host] int32 [B], 1 <= lens[b] <= Lmax
 *   speaker_ids [host] int32 [B] or NULL
 *   style_mel   [dev]  fp32 [B][style_frames][80] or NULL (GST models only)
 *   out         [dev]  fp32 [B][Lmax][256], every sentence encoded at its own length, rows past
 *                      lens[b] zero. */
tts_status tts_tacotron_encode(tts_tacotron* t, const int32_t* ids, const int32_t* lens, int B, int Lmax,
                               const int32_t* speaker_ids, const float* style_mel, int style_frames, float* out,
                               void* stream);

/* Replaces Decoder.inference (layers/tacotron.py:439-470) for a padded batch with per-sentence
 * batch-1 semantics (the reference's stop rule is batch-1, :464-469):
 *   enc [dev] fp32 [B][Lmax][256]; lens [host] int32 [B] (>= 1)
 *   mel [dev] fp32 [B][steps_cap*r][80]; stop [dev] fp32 [B][steps_cap] (sigmoid stop token);
 *   align [dev] fp32 [B][steps_cap][Lmax] or NULL; n_steps [host] int32 [B] out.
 * steps_cap >= max_steps + 1 (the reference stops once t > max_decoder_steps). */
tts_status tts_tacotron_decode(tts_tacotron* t, const float* enc, const int32_t* lens, int B, int Lmax,
                               int max_steps, int steps_cap, float* mel, float* stop, float* align,
                               int32_t* n_steps, void* stream);

/* Replaces PostCBHG + last_linear + sigmoid (layers/tacotron.py:246-259, models/tacotrongst.py:43-45,
 * 77-78): mel [dev] fp32 [B][Tmax][80], T [host] int32 [B] -> linear [dev] fp32 [B][Tmax][1025]
 * (rows past T[b] zero). */
tts_status tts_tacotron_postnet(tts_tacotron* t, const float* mel, const int32_t* T, int B, int Tmax,
                                float* linear, void* stream);

tts_status tts_tacotron_last_timing(tts_tacotron* t, float* loop_ms, int* steps_run);

/* Which implementation ran the last tts_tacotron_decode (no reference counterpart): *resident = 1
 * for the resident single-launch decoder (each XCD holds the step weights on its 32 compute units
 * and decodes up to 4 sentences; hand-offs stay inside the XCD), 0 for the per-step multi-launch
 * hipGraph path.  The resident path serves B <= 32, Lmax <= 256, r <= 6, max_steps <= 1000 under
 * config_tacotron_gst.json's attention (sigmoid norm, forward attention without the eval mask, no
 * transition agent / location / windowing) on a GPU with >= 256 compute units; TTS_RESIDENT=0 in
 * the environment at tts_tacotron_create disables it.  A resident run whose hand-off wait timed
 * out re-runs the batch on the multi-launch path (reported 0). */
tts_status tts_tacotron_last_path(tts_tacotron* t, int* resident);

/* Measurement only: re-runs the last resident tts_tacotron_decode batch with phase timers and
 * returns the mean microseconds per decoder step of each phase on compute units 0 (the attention
 * leader of sentence 0) and 1 (a non-leader) of XCD 0: us[0..15] and us[16..31] (n >= 32):
 * 0 wait prenet-1 + continue flags, 1 prenet-2 rows + gather, 2 attention-GRU unit + gather, 3 query
 * rows + gather, 4 energies / weights / context partial, 5 leader: slice sums + publish, 6 gather
 * contexts, 7 alignment + project_to_decoder_in + gather, 8 decoder GRU 1 + gather, 9 GRU 2 +
 * gather, 10 mel rows + gather, 11 prenet-1 rows + stopnet; 12-15 split the compute (up to the
 * publish) out of 2, 8, 9 and 10. */
#define TTS_TACOTRON_RESIDENT_PHASES 16
tts_status tts_tacotron_resident_phases(tts_tacotron* t, float* us, int n);

/* Measurement only: mean duration (ms) of each decoder-step kernel over up to `reps` eager steps
 * of the last decode's batch, HIP events on the library stream, in launch order: prenet2,
 * attention GRU, query, attention, project_to_decoder_in, decoder GRU 1, decoder GRU 2, mel,
 * [prenet1 | stopnet]. */
#define TTS_TACOTRON_STEP_KERNELS 9
tts_status tts_tacotron_profile(tts_tacotron* t, int reps, float* kernel_ms, int n_kernels);

const char* tts_last_error(void);
const char* tts_version(void);

#ifdef __cplusplus
}
#endif
#endif /* TTS_HIP_H */

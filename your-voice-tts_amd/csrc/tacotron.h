// Kernels of the Tacotron / TacotronGST path (tacotron_kernels.hip) used by tacotron_api.hip.
#pragma once
#include "common.h"

namespace tts {

constexpr int T_DEC = 256;            // encoder width = attention / decoder GRU width (layers/tacotron.py:289-305)
constexpr int T_PRE1 = 256;           // decoder prenet widths (:283-287)
constexpr int T_PRE2 = 128;
constexpr int T_XA = T_PRE2 + T_DEC;  // attention-GRU input row [prenet | context]
constexpr int GRU_H = 128;            // CBHG / reference-encoder GRU width (:165-170, gst_layers.py:53-56)

// GRU over whole sequences, one workgroup per (sentence, direction) (bigru_kernel).
struct GruSeqArgs {
    const float* xi;   // [B][Tmax][ndir * 384] input projections W_ih x + b_ih, gate rows r, z, n
    const int* T;      // [B] steps per sentence (0 = idle)
    int Tmax, ndir;
    const float* Whh;  // [ndir][384][128] reference layout
    const float* bhh;  // [ndir][384]
    float* out;        // [B][Tmax][out_ld], direction d at column d * 128 (may be null)
    int out_ld;
    const float* add1; // [B][add_ld] (may be null): out = (h + add1) + add2
    const float* add2;
    int add_ld;
    float* h_last;     // [B][ndir][128] final state (may be null)
};
hipError_t launch_bigru(const GruSeqArgs& a, int B, hipStream_t s);

// Decoder._init_states + Attention.init_states (layers/tacotron.py:336-357, common_layers.py:139-161).
struct TInitArgs {
    int B, Lcap, nmel;
    const int* lens;
    const float* att_init;  // [256] attention_rnn_init
    const float* dec_init;  // [2][256] decoder_rnn_inits
    const float* mem_init;  // [nmel] memory_init
    float* h_att;           // step 0 reads the parity-1 slots of h_att / h1 / h2
    float* h1;
    float* h2;
    int64_t h_pstride;
    float* xa;              // [.][T_XA], parity-0 context part zeroed
    float* mem;
    float *alpha, *att_w, *att_cum, *u;
    int *win_idx, *nidx;
    float* tail;
    int *flag1, *count, *done, *n_steps, *state;
};
hipError_t launch_tacotron_init(const TInitArgs& a, hipStream_t s);

// ReferenceEncoder Conv2d(3x3, stride 2, pad 1) + BatchNorm2d(eval, folded) + ReLU
// (layers/gst_layers.py:35-65).  in [B][Cin][H][W]; out [B][Cout][Ho][Wo], or with seq_layout
// the GRU input layout [B][Ho][Cout * Wo] (the transpose(1, 2) + view of :67-72).
hipError_t launch_gst_conv2d(const float* in, int Cin, int H, int W, const float* Wt, const float* scale,
                             const float* shift, int Cout, float* out, int seq_layout, int B, hipStream_t s);
// StyleTokenLayer + MultiHeadAttention (gst_layers.py:88-168): h [B][128] -> out [B][256].
hipError_t launch_style_attention(const float* h, const float* tokens, const float* Wq, const float* Wk,
                                  const float* Wv, float* out, int B, hipStream_t s);
// out[b][:] = table[ids[b]][:] (speaker embedding rows)
hipError_t launch_gather_rows(const float* table, const int* ids, int width, float* out, int B, hipStream_t s);
// logical weights [257][nmel + 256] of the [prenet L1 | stopnet] GEMM over x = [mel out | decoder out]:
// rows n < 256 = [W1[n] | 0], row 256 = [w_stop[256:] | w_stop[:256]] (stopnet input is
// cat([decoder_output, output]), layers/tacotron.py:388); biases [b1 | b_stop].
hipError_t fold_pre1_stop(const float* W1, const float* b1, const float* ws, const float* bs, int nmel, float* Wf,
                          float* bf, hipStream_t s);
hipError_t launch_fill_int(int* p, int n, int v, hipStream_t s);

}  // namespace tts

namespace tts {

// Resident decoder for TacotronGST / Tacotron (tacotron_resident.hip): the whole decoder loop of
// Decoder.inference (layers/tacotron.py:439-470) as ONE launch of 256 workgroups (one per CU).
// Each XCD runs its own group of up to TR_SPX sentences with a full copy of the step weights held
// on chip by its 32 CUs (6.7 MB per XCD: 106 VGPRs per thread); every hand-off stays inside the
// XCD.  Scope: the fast attention configuration (sigmoid norm, forward attention without the eval
// mask, no location / windowing / transition agent), memory_size == r, B <= 32, L <= 256,
// nmel <= 512, max_steps <= 1000.
constexpr int TR_CUS = 256, TR_THREADS = 512, TR_WAVES = TR_THREADS / 64;
constexpr int TR_SPX = 4;                    // sentences per XCD group
constexpr int TR_GROUPS = 8;                 // XCD groups
constexpr int TR_RANKS = 32;                 // CUs per group doing work
constexpr int TR_CPS = TR_RANKS / TR_SPX;    // attention CUs per sentence (positions split 8 ways)
constexpr int TR_PPC = 32;                   // encoder positions per attention CU (L <= 256)
constexpr int TR_LMAX = TR_CPS * TR_PPC;
constexpr int TR_NMEL_MAX = 512;
constexpr int TR_STATUS_PLACEMENT = 50;      // an XCD holds fewer than TR_RANKS workgroups
constexpr int TR_PHASES = 16;                // phase timers (tts_tacotron_resident_phases)

struct TResArgs {
    // weights, reference layouts (rows picked per XCD rank at run time)
    const float *a_wih, *a_whh, *a_bih, *a_bhh;  // attention_rnn [768][384], [768][256], [768], [768]
    const float *g_wih[2], *g_whh[2], *g_bih[2], *g_bhh[2];  // decoder_rnns [768][256] ...
    const float *w_proj, *b_proj;                // project_to_decoder_in [256][512], [256]
    const float *w_mel, *b_mel;                  // proj_to_mel [nmel][256], [nmel]
    const float *w_pre1, *b_pre1;                // prenet layer 0 [256][nmel], [256]
    const float *w_pre2, *b_pre2;                // prenet layer 1 [128][256], [128]
    const float* w_q;                            // query_layer [128][256]
    const float *v, *v_b;                        // attention v [128], [1]
    const float *w_stop, *b_stop;                // stopnet [256 + nmel], [1]
    int B, nmel, Lcap, Lalign, max_steps, hist_cap;
    const int* lens;     // [B] (device)
    const float* enc;    // [B][Lcap][256]
    const float* Pt;     // [B][128][Lcap]
    // initial state: the multi-launch buffers after launch_tacotron_init + the prenet go step
    const float *pre1, *h_att, *h1, *h2;  // pre1 [B][256]; step 0 reads slot 1 of h_att / h1 / h2
    int64_t h_pstride;
    const float* alpha;  // [B][Lcap]
    float *mel_hist, *stop_hist, *align_hist;  // [B][hist_cap][nmel], [B][hist_cap], [B][hist_cap][Lalign]
    int *done, *n_steps;
    unsigned long long* gran;  // tres_granules() granules (zeroed at create)
    int* status;               // 0 ok; TR_STATUS_PLACEMENT; else the id of the wait that timed out
    unsigned salt;             // per launch, 18 bits
    long long timeout_ticks;
    int first_sleep;  // s_sleep(1) count before a hand-off's first poll (TTS_TACO_FIRST_SLEEP)   // wall_clock64 ticks per wait
    long long* prof;           // null, or [2][TR_PHASES] phase ticks of CUs 0 and 1 of XCD 0 (measurement)
};
size_t tres_granules();
size_t tres_smem_bytes();
hipError_t tres_prepare();
hipError_t launch_tacotron_resident(const TResArgs& a, hipStream_t s, bool* launched);

}  // namespace tts

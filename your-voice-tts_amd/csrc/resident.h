// Resident (persistent) decoder for batch-1 synthesis: the whole decoder loop of
// Decoder.inference (layers/tacotron2.py:249-285) as ONE launch whose 256 workgroups (one per
// compute unit) keep every step weight on chip — 16 gate rows of both LSTMs per CU (the
// attention LSTM's in VGPRs, the decoder LSTM's recurrent/attention half in LDS, its context
// half in VGPRs) plus a prenet-2 row, a query row and one mel row (LDS).
// A step then streams no weights from HBM; its cost is the six dependent hand-offs
//   pre1 -> prenet2 -> h_att -> query -> [attention] -> ctx -> h_dec -> pre1
// of which pre1, prenet2, query and ctx stay inside one XCD: every XCD computes its own copy of
// the folded prenet-1 rows + stopnet (round 4: those 1.5 MB of rows are read from the XCD's L2
// every step, prefetched during the context and h_dec gathers; the register file and LDS are full), prenet-2,
// the query and the attention step (one attention CU per XCD; identical results), so only the
// two LSTM outputs cross XCDs.  Hand-offs are 8-byte {tag, value} granules (agent-scope relaxed
// atomics, sc1: the hand-off form that needs no fences, MI355X_MICROARCH.md "Valid forms").
// Every wait is bounded: a wave that does not see its data within the timeout flags an error
// and the grid drains.
//
// Scope: B = 1, L <= 256, nmel <= 256 (one mel row per CU; r <= 3), every Tacotron2 attention
// configuration (common_layers.py:107-256), in two forms:
//  - the synthesis configuration of synthesize.py:86 (forward attention + eval mask, sigmoid norm,
//    no location / windowing / transition agent — attention_uses_epart()): one attention CU per XCD
//    evaluates only the <= 15 positions the mask can keep (resident_decoder_kernel<., false>);
//  - every other configuration, among them Synthesizer.tts()'s (server/synthesizer.py:46-66 with
//    config_tacotron2.json: forward attention, sigmoid, mask off) and the constructor default
//    (location-sensitive + softmax, models/tacotron2.py:17,23): the attention of each XCD is spread
//    over its 32 CUs (resident_decoder_kernel<., true>).  CU rank k owns positions k + 32 w (one
//    per wave w) and context channels [16 k, 16 k + 16): energies (+ location features) of its
//    positions -> XCD-local publish -> every CU gathers all L energies and evaluates the
//    normalisation / windowing / forward attention / mask over them identically in every wave ->
//    the context of its 16 channels -> the existing context hand-off.  Reads its initial state from, and leaves its final
// state in, the multi-launch path's buffers (same slots), so continuous mode and profiling
// interoperate.
#pragma once
#include "decoder.h"

namespace tts {

constexpr int RES_CUS = 256;
constexpr int RES_THREADS = 512;
constexpr int RES_WAVES = RES_THREADS / 64;
constexpr int RES_LMAX = 256;

// granule slots (u64 {tag << 32 | float bits}) per step parity
// (GR_PRE2X: per-XCD prenet-2 vectors, [8 XCDs][256], written and read inside one XCD; GR_SETUP:
// each CU's XCD id, parity 0 only)
// GR_QX: per-XCD query half-rows [8][128 rows][2]; GR_CTXX: per-XCD context + tail [8][528];
// GR_P1X: per-XCD prenet-1 rows + continue flag [8][264] (slot 256 = flag).
// GR_EX: per-XCD attention energies [8][RES_LMAX] (general attention form: each CU of the XCD
// publishes the energies of its positions, every CU gathers all L).
constexpr int GR_HATT = 576, GR_HDEC = 2304, GR_PRE2X = 3328, GR_SETUP = 5376, GR_QX = 5632, GR_CTXX = 7680,
              GR_CTXX_STRIDE = ENC + 16, GR_P1X = 11904, GR_P1X_STRIDE = PRE + 8, GR_EX = GR_P1X + 8 * GR_P1X_STRIDE,
              GR_TOTAL = GR_EX + 8 * 256;
constexpr int RES_MIN_CUS_PER_XCD = 32;  // 8 XCDs x 32: query rows 4 per CU, prenet-1/2 rows 8 per CU
static_assert(RES_MIN_CUS_PER_XCD * 8 >= PRE, "at most one prenet row per wave");
constexpr int RES_STATUS_PLACEMENT = 50;  // status: an XCD holds fewer than RES_MIN_CUS_PER_XCD workgroups
constexpr int RES_PLACEMENT_RETRIES = 3;  // placement failures in a row before a handle stops trying
// the failure code of launch `salt` from its status word (salt << 8 | code; anything else: none)
inline int res_status_code(int word, unsigned salt) {
    return ((unsigned)word >> 8) == salt ? (word & 0xFF) : 0;
}
// next per-launch salt (18 bits, never 0); *wrapped: tags and status words of launches 2^18 back
// could match again, the caller clears its granules once
inline unsigned res_next_salt(unsigned salt, bool* wrapped) {
    salt = (salt + 1) & 0x3FFFF;
    *wrapped = salt == 0;
    return salt == 0 ? 1u : salt;
}

struct ResWeights {
    float4* wa;   // [256 CU][14 i4][512 thr]   attention LSTM rows over [prenet | ctx | h_att]
    float4* wdl;  // [256 CU][16 i4][16 row][32 ks]  decoder LSTM rows over [h_att | h_dec] (LDS image)
    float4* wdc;  // [256 CU][4 i4][512 thr]    decoder LSTM rows over ctx
    float* wf;    // folded rows [nrows][1536] = [mel | W1 W_mel (prenet-1) | stop] over [h_dec | ctx],
                  // reference layout: mel row c -> LDS of CU c; prenet-1 rows and the stop row per XCD
    float* bf;    // [nrows] folded biases
    float* ba;    // [256][16] attention LSTM bias (b_ih + b_hh), logical row g*4 + u
    float* bd;    // [256][16] decoder LSTM bias
    float* w2;    // prenet layer-2 weight, reference layout [256][256] (rows picked per XCD rank)
    float* wq;    // query_layer weight, reference layout [128][1024] (rows picked per XCD rank)
    float* b2;    // [256] prenet layer-2 bias (the BatchNorm prenet's folded shift; zeros otherwise)
};

// general attention form: configuration bits (ResArgs::gen; 0 = the synthesis-configuration form)
constexpr int GEN_ON = 1, GEN_SOFTMAX = 2, GEN_FORWARD = 4, GEN_MASK = 8, GEN_TA = 16, GEN_LOCATION = 32,
              GEN_WINDOW = 64;

struct ResArgs {
    ResWeights w;
    int gen;                  // GEN_* bits (general attention form) or 0
    const float* ta_w;        // transition agent [ENC + HATT] and bias [1] (GEN_TA)
    const float* ta_b;
    const float* att_w0;      // initial attention_weights / attention_weights_cum [Lcap] (GEN_LOCATION)
    const float* att_cum0;
    const int* win0;          // initial win_idx (GEN_WINDOW)
    const float* loc_conv;    // location_conv weight, packed [NLOC][2][32] (taps 31 + a zero)
    const float* loc_dense;   // location_dense weight [ADIM][NLOC] (reference layout)
    int L, Lcap, nmel, nrows, max_steps, hist_cap, Lalign;
    long long timeout_ticks;  // wall_clock64 ticks per wait
    unsigned salt;            // per-launch tag salt (18 bits): no granule of an earlier launch matches
    const float* v;
    const float* v_b;
    const float* Pt;   // [ADIM][Lcap] (sentence 0)
    const float* enc;  // [Lcap][ENC]
    // state, multi-launch layout (B = 1): step 0 reads slot 1 of h_att / h_dec and xa slot 0;
    // the last step n-1 leaves h in slot (n-1)&1 and ctx in xa slot 1-((n-1)&1)
    float* h_att;
    float* c_att;
    float* h_dec;
    float* c_dec;
    float* xa;
    int64_t hps, xps;
    float* pre1;  // relu(W1 mem): read at step 0, rewritten every step (next step's)
    const float* alpha;
    const int* nidx;
    const float* u;
    const int* flag1;
    const int* count;
    int* done;
    int* n_steps;
    float* mel_hist;
    float* stop_hist;
    float* align_hist;
    unsigned long long* gran;  // [2][GR_TOTAL], zeroed before every launch
    int* status;               // [0]: 0 ok, else the id of the wait that timed out
    // s_sleep(4) counts (~0.12 us each) before the first poll of a gather: a poll storm from every CU
    // slows the hand-off it waits for (device-wide h_att / h_dec; XCD-local pre1, prenet-2, context)
    int sleep_hatt, sleep_hdec, sleep_p1, sleep_pre2, sleep_ctx;
    int sleep_q, sleep_e;  // s_sleep(1) counts: the query gather, the general form's energy gather
    long long* prof;           // null, or RES_PROF_LL: [2][RES_PHASES] wall-clock ticks summed over steps
                               // per phase (CU 0, attention CU), then the event trace — measurement only
    int prof_marks;            // with prof: also the per-phase marks (they perturb the two CUs that take them)
};
constexpr int RES_PHASES = 16;
// profiling re-run only: prof also holds [256 CU][RES_TRACE_STEPS][RES_TRACE_EV] event ticks
// (P1, B1, h_att published, B3, B4, h_dec published, B6, pre1 row published, query row published;
// attention CUs: A1 (query gathered), A2 (candidate energies), context published)
constexpr int RES_TRACE_STEPS = 64, RES_TRACE_EV = 12;
constexpr size_t RES_PROF_LL = 2 * RES_PHASES + (size_t)RES_CUS * RES_TRACE_STEPS * RES_TRACE_EV;

// Pack the reference-layout weights (device pointers) into ResWeights (allocated by the caller,
// sizes from resident_weight_floats).
struct ResSrc {
    const float *a_wih, *a_whh, *a_bih, *a_bhh;  // attention_rnn [4096][768], [4096][1024]
    const float *d_wih, *d_whh, *d_bih, *d_bhh;  // decoder_rnn [4096][1536], [4096][1024]
    const float* w_pre2;                         // prenet layer 2 weight [256][256]
    const float* b_pre2;                         // its bias [256] or null (no bias)
    const float* w_q;                            // query_layer [128][1024]
    const float *wf, *bf;                        // folded [nrows][1536] + [nrows]
    int nrows;
};
void resident_weight_floats(size_t* wa, size_t* wdl, size_t* wdc);
hipError_t resident_pack(const ResSrc& src, const ResWeights& w, hipStream_t s);
// location_conv.weight [NLOC][2][KLOC] -> ResArgs::loc_conv [2][NLOC][32] (2 * NLOC * 32 floats)
hipError_t resident_pack_location(const float* w, float* out, hipStream_t s);
size_t resident_smem_bytes();
hipError_t resident_prepare();
// co-residency guaranteed or nothing launched (*launched = false): common.h launch_persistent
hipError_t launch_resident(const ResArgs& a, hipStream_t s, bool* launched);

// ---- resident decoder for batches of 2..RB_MAXB sentences (resident_batch.hip): the same
// weight-stationary design with both LSTMs' rows in registers and the batch's activations in LDS
constexpr int RB_MAXB = 4;  // per launch (larger requests: consecutive launches of <= RB_MAXB)
struct ResBatchArgs {
    int B, gen;                // sentences, GEN_* bits (resident_batch_supports)
    int L[RB_MAXB];            // encoder lengths (2..RES_LMAX)
    int Lcap, nmel, nrows, max_steps, hist_cap, Lalign;
    long long timeout_ticks;
    unsigned salt;
    const float4* wa;          // [256 CU][28][256 threads] 4 gates per k, attention LSTM (resident_batch_pack)
    const float4* wd;          // [256 CU][40][256 threads] decoder LSTM
    const float *w2, *b2, *wq, *wf, *bf, *ba, *bd;  // ResWeights' reference-layout rows and biases
    const float* v;
    const float* v_b;
    const float* Pt;           // [B][ADIM][Lcap]
    const float* enc;          // [B][Lcap][ENC]
    float *h_att, *c_att, *h_dec, *c_dec, *xa;  // multi-launch state layout ([2][Bcap][.] by parity)
    int64_t hps, xps;
    const float* pre1;         // [B][PRE] step-0 prenet layer 1
    const float* alpha;        // [B][Lcap]
    const int* nidx;
    const float* u;
    const int* flag1;
    const int* count;
    int* done;
    int* n_steps;
    float* mel_hist;           // [B][hist_cap][nmel]
    float* stop_hist;          // [B][hist_cap]
    float* align_hist;         // [B][hist_cap][Lalign]
    unsigned long long* gran;  // resident_batch_granules() slots
    int* status;
    int sleep_hatt, sleep_hdec, sleep_pre2, sleep_ctx;  // s_sleep(4) counts before a gather's first poll (TTS_RB_SLEEP_*)
    long long* prof;           // [256 CU][4 waves][RB_PROF_SLOTS] phase clocks (TTS_RB_PROF=1), else null
};
constexpr int RB_PROF_SLOTS = 26;  // [0, 13) phase sums, [13, 19) clocks at step RB_PROF_T, [20, 24) attention sub-phases, [25] steps
constexpr int RB_PROF_T = 150;
void resident_batch_weight_floats(size_t* wa, size_t* wd);
size_t resident_batch_granules();
hipError_t resident_batch_pack(const ResSrc& src, float4* wa, float4* wd, hipStream_t s);
hipError_t resident_batch_prepare();
bool resident_batch_supports(int gen);
hipError_t launch_resident_batch(const ResBatchArgs& a, hipStream_t s, bool* launched);

}  // namespace tts

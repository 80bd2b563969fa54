// Host runtime of the decoder: weight repacking/folding, workspace, hipGraph-captured step loop.
//
// One decoder step = 6 launches on the library's own stream:
//   prenet L2 (sgemm relu) -> attention LSTM (sgemm + LSTM epilogue) -> query (sgemm)
//   -> attention (1 WG / sentence) -> decoder LSTM (sgemm + LSTM epilogue)
//   -> fused [mel projection | next step's prenet L1 | stopnet + stop rule] (sgemm).
// Prenet L1 and the stopnet are folded into the mel projection at load time (W1 W_mel and
// w_stop W_mel, fp64), so the reference's mel -> prenet -> ... chain loses two dependent launches.
// Ping-pong activation buffers are bound statically per step parity: three graphs are captured
// per (B, Lmax, max_steps) — one even step, one odd step, and a CHUNK-step run starting even.
// The step index and active count live in device memory in two parity slots {step, n_active}:
// a step reads its own slot and the stop rule writes the other, so no launch ever races on it.
// The host synchronises only at chunk boundaries: the first chunk is the reference's lower
// bound on the step count (min(2L+22, max_steps) per sentence, layers/tacotron2.py:268-277).
#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "decoder.h"
#include "resident.h"
#include "sgemm.h"

using namespace tts;

namespace {
struct Graphs {
    hipGraphExec_t step[2] = {nullptr, nullptr};
    hipGraphExec_t chunk = nullptr;
};
constexpr int CHUNK = 8;
}  // namespace

struct tts_decoder {
    tts_decoder_config cfg{};
    int nmel = 80;
    hipStream_t stream = nullptr;
    hipEvent_t ev_in = nullptr, ev_out = nullptr, ev_t0 = nullptr, ev_t1 = nullptr;
    hipEvent_t ev_sync = nullptr;  // spin_sync (runtime.hip)
    std::vector<void*> allocs;
    // packed GEMM weights + logical biases
    float *b_pre1 = nullptr, *b_pre2 = nullptr;  // prenet_type "bn": the folded shifts (else null)
    float *W_pre1 = nullptr, *W_pre2 = nullptr, *W_att = nullptr, *b_att = nullptr, *W_q = nullptr;
    float *W_dec = nullptr, *b_dec = nullptr, *W_melf = nullptr, *b_melf = nullptr;
    // reference-layout small weights
    float *v = nullptr, *v_b = nullptr, *ta_w = nullptr, *ta_b = nullptr, *loc_conv = nullptr, *loc_dense = nullptr;
    float *W_in = nullptr, *att_init = nullptr, *dec_init = nullptr, *go = nullptr;
    // workspace
    int Lcap = 0, Bcap = 0, hist_cap = 0;
    float *enc = nullptr, *Pt = nullptr, *h_att = nullptr, *c_att = nullptr, *h_dec = nullptr, *c_dec = nullptr;
    float *xa = nullptr, *mem = nullptr, *pre1 = nullptr, *q = nullptr, *epart = nullptr;
    // fragment-order mirrors (common.h: frag_idx, ntf m-tiles) of the GEMM inputs for batches
    // above 16: written beside the row-major buffers by their producers, read by the 4-wave
    // batched GEMM (sgemm.h: Seg::pf).  Null when max_batch <= 16.
    int ntf = 0;
    float *xaf = nullptr, *hattf = nullptr, *hdecf = nullptr, *pre1f = nullptr;
    int res_gen = 0;              // resident decoder form: 0 = synthesis configuration, else GEN_* bits
    float* loc_conv_p = nullptr;  // location_conv packed for the general resident form
    bool fast_attention = false;  // attention_uses_epart(): the synthesis configuration's attention
                                  // launch (attention_fm_kernel) and the resident decoder
    float* locf = nullptr;        // location_attn: [Bcap][NLOC][Lcap] location features of the next step
    // resident (persistent, one launch per sentence) batch-1 decoder, resident.h
    bool resident = false;
    ResWeights rw{};
    unsigned long long* gran = nullptr;  // [2][GR_TOTAL] granules, then int status[4]
    long long res_ticks = 0;
    unsigned res_salt = 0;
    float *alpha = nullptr, *att_w = nullptr, *att_cum = nullptr, *u = nullptr, *tail = nullptr;
    int *lens = nullptr, *win_idx = nullptr, *nidx = nullptr, *flag1 = nullptr, *count = nullptr, *done = nullptr;
    int *n_steps = nullptr, *state = nullptr;  // state: [2][2] = {step, n_active} per parity
    float *mel_hist = nullptr, *stop_hist = nullptr, *align_hist = nullptr;
    int* host_flags = nullptr;  // pinned coherent: [0, 3) flags, [3] read-back sequence, [4, 4 + 64) step counts
    int rb_seq = 0;             // the resident run's read-back sequence number (host_flags[3])
    // tts_synth_run: work enqueued behind a resident launch before the host waits for it (the
    // postnet, reading the device step counts); hook_ran reports that it was enqueued
    void (*post_hook)(void*, hipStream_t) = nullptr;
    void* post_ctx = nullptr;
    bool hook_ran = false;
    // tts_synth_run (decoder_set_pipeline_io): device length array, one extra status word to read
    // back, the speculative Griffin-Lim frame-count clamp target
    const int* io_lens = nullptr;
    const int* io_rb_src = nullptr;
    int* io_rb_dst = nullptr;
    int* io_clamp = nullptr;
    int io_clamp_max = 0;
    // relu(W_pre1 go): the step-0 prenet layer 1 of a fresh batch-1 resident run, copied by
    // decoder_init instead of a GEMM launch per sentence (computed by the first such run)
    float* pre1_go = nullptr;
    bool pre1_go_ok = false;
    const float* last_enc_direct = nullptr;  // the last direct run's encoder output (profiling re-runs)
    int last_len_direct = 0;                 // ... and its length (the device copy it read may be reused)
    std::vector<long long> res_trace;        // the last tts_decoder_resident_phases run's event trace
    std::map<std::tuple<int, int, int>, Graphs> graphs;
    float last_ms = 0.f;
    bool pipeline = false;  // tts_synth_run: work on the caller's stream
    // tts_synth_run: leave mel / stop / alignments in the histories (decoder_histories) instead of
    // copying them out (the postnet reads the mel history in place)
    bool keep_hist = false;
    int last_steps = 0;
    int last_B = 0, last_Lmax = 0, last_max_steps = 0, last_first = 0;
    int last_steps_done = 0;  // steps of the last batch-1 run (continuous mode), 0 otherwise
    int last_resident = 0;    // the last run used the resident decoder
    int res_timeouts = 0;     // resident runs that timed out a hand-off and re-ran multi-launch
    int res_place_fails = 0;  // consecutive resident runs that stopped on a placement failure
    // resident decoder for batches of 2..RB_MAXB sentences per launch (resident_batch.hip)
    bool rbatch = false;
    int rb_gen = 0;
    float4 *rb_wa = nullptr, *rb_wd = nullptr;
    long long* rb_prof = nullptr;           // TTS_RB_PROF=1 phase clocks
    unsigned long long* rb_gran = nullptr;  // resident_batch_granules() slots, then int status[4]
    unsigned rb_salt = 0;
    int rb_place_fails = 0;
    ResArgs last_ra{};
    InitArgs last_init{};
};

namespace {

// the largest batch the resident batch decoder takes (consecutive launches of <= RB_MAXB): two
// launches of 4 (2 x 16.6 us per step, round 6) beat the multi-launch step (~44 us at any batch up
// to 64); three do not.  TTS_RB_MAX overrides.
int rb_max_batch() {
    static const int v = [] {
        const char* e = getenv("TTS_RB_MAX");
        return e && e[0] ? std::max(0, atoi(e)) : 2 * RB_MAXB;
    }();
    return v;
}

template <typename T>
tts_status dmalloc(tts_decoder* d, T** p, size_t n) {
    void* q = nullptr;
    TTS_HIP(hipMalloc(&q, n * sizeof(T) + 16));
    d->allocs.push_back(q);
    *p = static_cast<T*>(q);
    return TTS_OK;
}

struct WeightMap {
    std::unordered_map<std::string, std::pair<const float*, int64_t>> m;
    const float* get(const std::string& k, int64_t numel) const {
        auto it = m.find(k);
        if (it == m.end()) { set_error("missing weight " + k); return nullptr; }
        if (it->second.second != numel) {
            set_error("weight " + k + " has " + std::to_string(it->second.second) + " elements, expected " +
                      std::to_string(numel));
            return nullptr;
        }
        return it->second.first;
    }
};

tts_status copy_weight(tts_decoder* d, float** dst, const float* src, size_t n, hipStream_t s) {
    tts_status st = dmalloc(d, dst, n);
    if (st) return st;
    TTS_HIP(hipMemcpyAsync(*dst, src, n * sizeof(float), hipMemcpyDeviceToDevice, s));
    return TTS_OK;
}

// The batched GEMMs read fragment mirrors above 16 sentences (TTS_FRAG=0: row-major always).
bool frag_on(const tts_decoder* d, int B) {
    static const bool off = [] {
        const char* e = std::getenv("TTS_FRAG");
        return e && e[0] == '0';
    }();
    return d->xaf && B > 16 && !off;
}

// Mirrors of the state a run starts from (after launch_decoder_init): both parities of xa, h_att
// and h_dec (pre1 is mirrored by the prenet launch that writes it).
tts_status enqueue_frag_sync(tts_decoder* d, int B, hipStream_t s) {
    const int64_t hps = (int64_t)d->Bcap * HATT, xps = (int64_t)d->Bcap * XA;
    const int64_t fh = (int64_t)d->ntf * 16 * HATT, fx = (int64_t)d->ntf * 16 * XA;
    for (int p = 0; p < 2; ++p) {
        struct { const float* src; int64_t ld; int K; float* dst; } jobs[3] = {
            {d->xa + p * xps, XA, XA, d->xaf + p * fx},
            {d->h_att + p * hps, HATT, HATT, d->hattf + p * fh},
            {d->h_dec + p * hps, HDEC, HDEC, d->hdecf + p * fh}};
        for (auto& j : jobs) TTS_HIP(frag_mirror(j.src, j.ld, B, j.K, j.dst, d->ntf, s));
    }
    return TTS_OK;
}

// Launches of one decoder step of parity p (0: even step, 1: odd step).  `ev` (optional, 7
// events) brackets every launch for tts_decoder_profile.
tts_status enqueue_step(tts_decoder* d, int B, int Lmax, int max_steps, int p, hipStream_t s,
                        hipEvent_t* ev = nullptr, int rule = 0) {
    int mark = 0;
#define MARK() \
    if (ev) TTS_HIP(hipEventRecord(ev[mark++], s));
    const int nmel = d->nmel;
    const int q = 1 - p;
    const int64_t hps = (int64_t)d->Bcap * HATT;  // ping-pong slot strides
    const int64_t xps = (int64_t)d->Bcap * XA;
    float* h_att_cur = d->h_att + p * hps;
    float* h_att_prev = d->h_att + q * hps;
    float* h_dec_cur = d->h_dec + p * hps;
    float* h_dec_prev = d->h_dec + q * hps;
    float* xa_cur = d->xa + p * xps;   // [prenet_t | ctx_{t-1}]
    float* ctx_cur = d->xa + q * xps + PRE;  // ctx_t (row stride XA)
    int* st_cur = d->state + 2 * p;
    // fragment mirrors of the same buffers (batches above 16)
    const bool fr = frag_on(d, B);
    const int64_t fh = (int64_t)d->ntf * 16 * HATT, fx = (int64_t)d->ntf * 16 * XA;
    const int64_t fchunk = (int64_t)d->ntf * 256;  // floats per 16-column chunk of a mirror
    float* hattf_cur = fr ? d->hattf + p * fh : nullptr;
    float* hattf_prev = fr ? d->hattf + q * fh : nullptr;
    float* hdecf_cur = fr ? d->hdecf + p * fh : nullptr;
    float* hdecf_prev = fr ? d->hdecf + q * fh : nullptr;
    float* xaf_cur = fr ? d->xaf + p * fx : nullptr;
    float* ctxf_cur = fr ? d->xaf + q * fx + (PRE / 16) * fchunk : nullptr;  // ctx_t: xa columns PRE..
    SGemmArgs g{};
    g.B = B;
    g.step = st_cur;
    g.done = d->done;
    g.out_par = -1;
    g.ntf = d->ntf;
    // 1) prenet layer 2 -> xa_cur[b][0:256]   (common_layers.py:77-83; dropout off in eval)
    {
        SGemmArgs a = g;
        a.seg[0] = Seg{d->pre1, PRE, PRE, fr ? d->pre1f : nullptr};
        a.nseg = 1;
        a.W = d->W_pre2; a.K = PRE; a.N = PRE; a.act = ACT_RELU; a.bias = d->b_pre2;
        a.out = xa_cur; a.ldo = XA;
        a.outf = xaf_cur; a.outf_k0 = 0;
        MARK();
        TTS_HIP(sgemm_launch(a, ROLE_PRENET, s));
    }
    // 2) attention LSTM: x = [prenet_t | ctx_{t-1}], h = h_att_{t-1}   (tacotron2.py:195-197)
    {
        SGemmArgs a = g;
        a.seg[0] = Seg{xa_cur, XA, XA, xaf_cur};
        a.seg[1] = Seg{h_att_prev, HATT, HATT, hattf_prev};
        a.nseg = 2;
        a.W = d->W_att; a.K = XA + HATT; a.N = 4 * HATT; a.bias = d->b_att;
        a.out = h_att_cur; a.ldo = HATT;
        a.outf = hattf_cur; a.outf_k0 = 0;
        a.cell = d->c_att; a.ldc = HATT;
        MARK();
        TTS_HIP(sgemm_launch(a, ROLE_ATT_LSTM, s));
    }
    // 3) processed query = query_layer(h_att_t) (common_layers.py:170/179) and, for the fast
    //    attention path, the energy partials v . tanh(q + P_j) over 16 dims per workgroup
    {
        QEArgs a{};
        a.Wq = d->W_q; a.h = h_att_cur; a.v = d->v; a.Pt = d->Pt; a.lens = d->lens; a.Lcap = d->Lcap;
        // every configuration: the energies as QE_TILES partials per position (with the location
        // term from the previous attention launch's features)
        a.energies = 1;
        a.locf = d->locf; a.loc_dense = d->loc_dense;
        a.q = d->q; a.epart = d->epart; a.step = st_cur;
        MARK();
        TTS_HIP(launch_query_energy(a, B, s));
    }
    // 4) attention (energies, norm, forward attention, context -> ctx_t)
    {
        AttnArgs a{};
        const tts_decoder_config& c = d->cfg;
        a.attn_norm = c.attn_norm; a.forward_attn = c.forward_attn; a.trans_agent = c.trans_agent;
        a.forward_attn_mask = c.forward_attn_mask; a.location_attn = c.location_attn; a.windowing = c.windowing;
        a.Lcap = d->Lcap; a.B = B; a.enc_dim = ENC; a.ctx_ld = XA; a.tail_rule = 0;
        a.v = d->v; a.v_b = d->v_b; a.ta_w = d->ta_w; a.ta_b = d->ta_b;
        a.loc_conv = d->loc_conv; a.loc_dense = d->loc_dense;
        a.q = d->q; a.Pt = d->Pt; a.enc = d->enc; a.lens = d->lens;
        a.h_att = h_att_cur;
        a.epart = d->epart; a.locf = d->locf;
        a.sstride = (int64_t)d->Bcap * d->Lcap; a.istride = d->Bcap;
        a.ctx_prev = xa_cur + PRE; a.h_att_prev = h_att_prev;
        a.alpha = d->alpha; a.att_w = d->att_w; a.att_cum = d->att_cum; a.u = d->u; a.win_idx = d->win_idx;
        a.nidx = d->nidx; a.tail = d->tail;
        a.ctx = ctx_cur;  // kernel writes ctx[b*XA + d]
        a.ctxf = fr ? d->xaf + q * fx : nullptr; a.ctxf_k0 = PRE; a.ntf = d->ntf;
        a.align_hist = d->align_hist; a.align_ldb = (int64_t)d->hist_cap * Lmax; a.Lalign = Lmax;
        a.hist_cap = d->hist_cap;
        a.step = st_cur; a.done = d->done;
        MARK();
        TTS_HIP(launch_attention(a, s));
    }
    // 5) decoder LSTM: x = [h_att_t | ctx_t], h = h_dec_{t-1}   (tacotron2.py:206-208)
    {
        SGemmArgs a = g;
        a.seg[0] = Seg{h_att_cur, HATT, HATT, hattf_cur};
        a.seg[1] = Seg{ctx_cur, XA, ENC, ctxf_cur};
        a.seg[2] = Seg{h_dec_prev, HDEC, HDEC, hdecf_prev};
        a.nseg = 3;
        a.W = d->W_dec; a.K = HATT + ENC + HDEC; a.N = 4 * HDEC; a.bias = d->b_dec;
        a.out = h_dec_cur; a.ldo = HDEC;
        a.outf = hdecf_cur; a.outf_k0 = 0;
        a.cell = d->c_dec; a.ldc = HDEC;
        MARK();
        TTS_HIP(sgemm_launch(a, ROLE_DEC_LSTM, s));
    }
    // 6) fused: mel = linear_projection([h_dec | ctx]) (tacotron2.py:214-217) -> history;
    //    prenet L1 of the next step; stop = sigmoid(stopnet([h_dec; mel])) + stop rule (:219-277)
    {
        SGemmArgs a = g;
        a.seg[0] = Seg{h_dec_cur, HDEC, HDEC, hdecf_cur};
        a.seg[1] = Seg{ctx_cur, XA, ENC, ctxf_cur};
        a.nseg = 2;
        a.W = d->W_melf; a.K = HDEC + ENC; a.N = nmel + PRE + 1; a.bias = d->b_melf;
        a.hist = d->mel_hist; a.ldh = (int64_t)d->hist_cap * nmel; a.hist_cap = d->hist_cap;
        MelFused& m = a.mf;
        m.nmel = nmel; m.pre1 = d->pre1; m.ldp = PRE;
        m.pre1f = fr ? d->pre1f : nullptr;
        m.stop_hist = d->stop_hist; m.stop_ldb = d->hist_cap;
        m.lens = d->lens; m.tail = d->tail; m.flag1 = d->flag1; m.count = d->count;
        m.done = d->done; m.n_steps = d->n_steps;
        m.state_next = d->state + 2 * q;
        m.stop_acc = d->state + 4;
        m.max_steps = max_steps;
        m.rule = rule;
        MARK();
        TTS_HIP(sgemm_launch(a, ROLE_MEL_FUSED, s));
    }
    MARK();
#undef MARK
    return TTS_OK;
}

tts_status build_graph(tts_decoder* d, int B, int Lmax, int max_steps, int first_parity, int steps,
                       hipGraphExec_t* out) {
    hipGraph_t g = nullptr;
    TTS_HIP(hipStreamBeginCapture(d->stream, hipStreamCaptureModeThreadLocal));
    tts_status st = TTS_OK;
    for (int i = 0; i < steps && st == TTS_OK; ++i)
        st = enqueue_step(d, B, Lmax, max_steps, (first_parity + i) & 1, d->stream);
    hipError_t e = hipStreamEndCapture(d->stream, &g);
    if (st) return st;
    TTS_HIP(e);
    TTS_HIP(hipGraphInstantiate(out, g, nullptr, nullptr, 0));
    TTS_HIP(hipGraphDestroy(g));
    return TTS_OK;
}

// Step-0 prenet layer 1 on the go frame (later steps get it from the fused mel launch; under
// teacher forcing every step runs it on the teacher frame in mem, `slot` = that step's state slot).
tts_status enqueue_prenet_go(tts_decoder* d, int B, hipStream_t s, int* slot = nullptr) {
    SGemmArgs a{};
    a.B = B;
    a.step = slot ? slot : d->state;
    a.out_par = -1;
    a.seg[0] = Seg{d->mem, d->nmel, d->nmel};
    a.nseg = 1;
    a.W = d->W_pre1; a.K = d->nmel; a.N = PRE; a.act = ACT_RELU; a.bias = d->b_pre1;
    a.out = d->pre1; a.ldo = PRE;
    if (frag_on(d, B)) { a.outf = d->pre1f; a.outf_k0 = 0; a.ntf = d->ntf; }
    TTS_HIP(sgemm_launch(a, ROLE_PRENET, s));
    return TTS_OK;
}

}  // namespace

namespace {
tts_status decoder_run(tts_decoder* d, const float* enc, const int32_t* lens, int B, int Lmax, int max_steps,
                       int steps_cap, float* mel, float* stop, float* align, int32_t* n_steps, void* stream, bool keep);
}

extern "C" {

tts_status tts_decoder_create(const tts_decoder_config* cfg, const tts_tensor* tensors, int n_tensors, void* stream,
                              tts_decoder** out) {
    TTS_CHECK(cfg && out && (tensors || n_tensors == 0), TTS_ERR_INVALID, "null argument");
    TTS_CHECK(cfg->r >= 1 && cfg->r <= 8, TTS_ERR_INVALID, "r must be in [1, 8]");
    TTS_CHECK(cfg->max_batch >= 1 && cfg->max_batch <= 64, TTS_ERR_UNSUPPORTED, "max_batch must be in [1, 64]");
    TTS_CHECK(cfg->max_len >= 2 && cfg->max_len <= (cfg->location_attn ? 512 : 1024), TTS_ERR_UNSUPPORTED,
              "max_len must be in [2, 1024] (512 with location attention)");
    TTS_CHECK(cfg->max_steps >= 1, TTS_ERR_INVALID, "max_steps must be >= 1");
    TTS_CHECK(cfg->attn_norm == 0 || cfg->attn_norm == 1, TTS_ERR_INVALID, "Unknown value for attention norm type");
    TTS_CHECK(!cfg->trans_agent || cfg->forward_attn, TTS_ERR_INVALID, "trans_agent requires forward_attn");
    auto* d = new tts_decoder();
    d->cfg = *cfg;
    d->nmel = 80 * cfg->r;
    hipStream_t s = static_cast<hipStream_t>(stream);
    tts_status st = TTS_OK;
    auto fail = [&](tts_status code) { tts_decoder_destroy(d); return code; };
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&d->ev_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&d->ev_out, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&d->ev_t0, hipEventReleaseToDevice) != hipSuccess ||
        hipEventCreateWithFlags(&d->ev_t1, hipEventReleaseToDevice) != hipSuccess ||
        hipEventCreateWithFlags(&d->ev_sync, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&d->host_flags), (4 + 64) * sizeof(int), hipHostMallocCoherent) != hipSuccess) {
        set_error("stream/event creation failed");
        return fail(TTS_ERR_HIP);
    }
    // the host polls host_flags[3] for ++rb_seq (from 1): a recycled pinned block could still hold
    // an earlier handle's sequence value, so the words start at zero
    std::memset(d->host_flags, 0, (4 + 64) * sizeof(int));
    WeightMap wm;
    for (int i = 0; i < n_tensors; ++i) wm.m[tensors[i].key] = {tensors[i].data, tensors[i].numel};
    const int nmel = d->nmel;
#define GW(var, key, n)                        \
    const float* var = wm.get(key, n);         \
    if (!var) return fail(TTS_ERR_INVALID);
    GW(pre0, "decoder.prenet.layers.0.linear_layer.weight", (int64_t)PRE * nmel);
    GW(pre1, "decoder.prenet.layers.1.linear_layer.weight", (int64_t)PRE * PRE);
    GW(a_wih, "decoder.attention_rnn.weight_ih", (int64_t)4 * HATT * XA);
    GW(a_whh, "decoder.attention_rnn.weight_hh", (int64_t)4 * HATT * HATT);
    GW(a_bih, "decoder.attention_rnn.bias_ih", 4 * HATT);
    GW(a_bhh, "decoder.attention_rnn.bias_hh", 4 * HATT);
    GW(wq, "decoder.attention_layer.query_layer.linear_layer.weight", (int64_t)ADIM * HATT);
    GW(win, "decoder.attention_layer.inputs_layer.linear_layer.weight", (int64_t)ADIM * ENC);
    GW(vw, "decoder.attention_layer.v.linear_layer.weight", ADIM);
    GW(vb, "decoder.attention_layer.v.linear_layer.bias", 1);
    GW(d_wih, "decoder.decoder_rnn.weight_ih", (int64_t)4 * HDEC * (HATT + ENC));
    GW(d_whh, "decoder.decoder_rnn.weight_hh", (int64_t)4 * HDEC * HDEC);
    GW(d_bih, "decoder.decoder_rnn.bias_ih", 4 * HDEC);
    GW(d_bhh, "decoder.decoder_rnn.bias_hh", 4 * HDEC);
    GW(pw, "decoder.linear_projection.linear_layer.weight", (int64_t)nmel * (HDEC + ENC));
    GW(pb, "decoder.linear_projection.linear_layer.bias", nmel);
    GW(sw, "decoder.stopnet.1.linear_layer.weight", HDEC + nmel);
    GW(sb, "decoder.stopnet.1.linear_layer.bias", 1);
    GW(ainit, "decoder.attention_rnn_init.weight", HATT);
    GW(goinit, "decoder.go_frame_init.weight", nmel);
    GW(dinit, "decoder.decoder_rnn_inits.weight", HDEC);
    const float *taw = nullptr, *tab = nullptr, *lcw = nullptr, *ldw = nullptr;
    if (cfg->trans_agent) {
        taw = wm.get("decoder.attention_layer.ta.weight", HATT + ENC);
        tab = wm.get("decoder.attention_layer.ta.bias", 1);
        if (!taw || !tab) return fail(TTS_ERR_INVALID);
    }
    if (cfg->location_attn) {
        lcw = wm.get("decoder.attention_layer.location_layer.location_conv.weight", NLOC * 2 * KLOC);
        ldw = wm.get("decoder.attention_layer.location_layer.location_dense.linear_layer.weight", ADIM * NLOC);
        if (!lcw || !ldw) return fail(TTS_ERR_INVALID);
    }
#undef GW
#define CK(x)                              \
    do {                                   \
        st = (x);                          \
        if (st) return fail(st);           \
    } while (0)
#define HK(x)                                                            \
    do {                                                                 \
        hipError_t _e = (x);                                             \
        if (_e != hipSuccess) return fail(hip_fail(_e, #x, __FILE__, __LINE__)); \
    } while (0)
    {
        AttnArgs probe{};
        probe.attn_norm = cfg->attn_norm; probe.forward_attn = cfg->forward_attn; probe.trans_agent = cfg->trans_agent;
        probe.forward_attn_mask = cfg->forward_attn_mask; probe.location_attn = cfg->location_attn;
        probe.windowing = cfg->windowing;
        probe.enc_dim = ENC;
        d->fast_attention = attention_uses_epart(probe);
        // the general resident form for every other configuration (resident.h); TTS_RESIDENT_GEN=0
        // keeps those on the multi-launch path (A/B, parity reference)
        const char* ge = getenv("TTS_RESIDENT_GEN");
        if (!d->fast_attention && !(ge && ge[0] == '0')) {
            d->res_gen = GEN_ON | (cfg->attn_norm == 0 ? GEN_SOFTMAX : 0) | (cfg->forward_attn ? GEN_FORWARD : 0) |
                         (cfg->forward_attn && cfg->forward_attn_mask ? GEN_MASK : 0) |
                         (cfg->forward_attn && cfg->trans_agent ? GEN_TA : 0) | (cfg->location_attn ? GEN_LOCATION : 0) |
                         (cfg->windowing ? GEN_WINDOW : 0);
        }
    }
    // prenet_type "bn" (common_layers.py:55-70, Decoder's Prenet(bias=False) layers/tacotron2.py:114):
    // each layer is Linear -> BatchNorm1d (eval: running statistics, eps 1e-5) -> ReLU, folded here
    // into the layer's weight plus a bias that every prenet consumer below adds
    const float *w_p0 = pre0, *w_p1 = pre1;
    if (wm.m.count("decoder.prenet.layers.0.bn.weight") || wm.m.count("decoder.prenet.layers.1.bn.weight")) {
        const int fan_in[2] = {nmel, PRE};
        const float* w_in[2] = {pre0, pre1};
        float* w_out[2] = {nullptr, nullptr};
        float* b_out[2] = {nullptr, nullptr};
        for (int l = 0; l < 2; ++l) {
            const std::string k = "decoder.prenet.layers." + std::to_string(l) + ".bn.";
            const float* g = wm.get(k + "weight", PRE);
            const float* be = wm.get(k + "bias", PRE);
            const float* mu = wm.get(k + "running_mean", PRE);
            const float* var = wm.get(k + "running_var", PRE);
            if (!g || !be || !mu || !var) return fail(TTS_ERR_INVALID);
            CK(dmalloc(d, &w_out[l], (size_t)PRE * fan_in[l]));
            CK(dmalloc(d, &b_out[l], PRE));
            HK(fold_linear_bn(w_in[l], nullptr, g, be, mu, var, PRE, fan_in[l], 1e-5f, w_out[l], b_out[l], s));
        }
        w_p0 = w_out[0]; w_p1 = w_out[1];
        d->b_pre1 = b_out[0]; d->b_pre2 = b_out[1];
    }
    // packed GEMM weights
    const int nfused = nmel + PRE + 1;
    {
        // the resident decoder needs one workgroup per CU on >= 256 CUs and one mel row per CU;
        // TTS_RESIDENT=0 disables it (multi-launch path for every batch)
        const char* env = getenv("TTS_RESIDENT");
        int dev = 0, ncu = 0, rate_khz = 0;
        if ((d->fast_attention || d->res_gen) && nmel <= RES_CUS && !(env && env[0] == '0') && hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu >= RES_CUS &&
            hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && rate_khz > 0 &&
            resident_prepare() == hipSuccess) {
            d->resident = true;
            d->res_ticks = (long long)rate_khz * 50;  // 50 ms per hand-off wait
            // fault injection for the timeout fallback test (TTS_DEC_WAIT_TICKS wall-clock ticks)
            if (const char* tk = getenv("TTS_DEC_WAIT_TICKS"); tk && tk[0]) d->res_ticks = std::max(1LL, atoll(tk));
        }
    }
    CK(dmalloc(d, &d->W_pre1, sgemm_packed_floats(PRE, nmel)));
    HK(sgemm_pack(w_p0, nmel, nullptr, 0, PRE, ROWMAP_IDENTITY, 0, d->W_pre1, s));
    CK(dmalloc(d, &d->W_pre2, sgemm_packed_floats(PRE, PRE)));
    HK(sgemm_pack(w_p1, PRE, nullptr, 0, PRE, ROWMAP_IDENTITY, 0, d->W_pre2, s));
    CK(dmalloc(d, &d->W_att, sgemm_packed_floats(4 * HATT, XA + HATT)));
    HK(sgemm_pack(a_wih, XA, a_whh, HATT, 4 * HATT, ROWMAP_LSTM, HATT, d->W_att, s));
    CK(dmalloc(d, &d->b_att, 4 * HATT));
    HK(sgemm_pack_bias(a_bih, a_bhh, 4 * HATT, ROWMAP_LSTM, HATT, d->b_att, s));
    CK(dmalloc(d, &d->W_q, sgemm_packed_floats(ADIM, HATT)));
    HK(sgemm_pack(wq, HATT, nullptr, 0, ADIM, ROWMAP_IDENTITY, 0, d->W_q, s));
    CK(dmalloc(d, &d->W_dec, sgemm_packed_floats(4 * HDEC, HATT + ENC + HDEC)));
    HK(sgemm_pack(d_wih, HATT + ENC, d_whh, HDEC, 4 * HDEC, ROWMAP_LSTM, HDEC, d->W_dec, s));
    CK(dmalloc(d, &d->b_dec, 4 * HDEC));
    HK(sgemm_pack_bias(d_bih, d_bhh, 4 * HDEC, ROWMAP_LSTM, HDEC, d->b_dec, s));
    {
        float *wf = nullptr, *bf = nullptr;  // folded logical matrix (temporary)
        HK(hipMalloc(&wf, sizeof(float) * nfused * (HDEC + ENC)));
        HK(hipMalloc(&bf, sizeof(float) * nfused));
        hipError_t e = fold_mel_weights(pw, pb, w_p0, d->b_pre1, sw, sb, nmel, HDEC + ENC, HDEC, wf, bf, s);
        if (e == hipSuccess) e = dmalloc(d, &d->W_melf, sgemm_packed_floats(nfused, HDEC + ENC)) ? hipErrorOutOfMemory
                                                                                                : hipSuccess;
        if (e == hipSuccess) e = sgemm_pack(wf, HDEC + ENC, nullptr, 0, nfused, ROWMAP_IDENTITY, 0, d->W_melf, s);
        if (e == hipSuccess) e = dmalloc(d, &d->b_melf, (nfused + 15) / 16 * 16) ? hipErrorOutOfMemory : hipSuccess;
        if (e == hipSuccess) e = sgemm_pack_bias(bf, nullptr, nfused, ROWMAP_IDENTITY, 0, d->b_melf, s);
        if (e == hipSuccess && d->resident) {
            size_t nwa, nwdl, nwdc;
            resident_weight_floats(&nwa, &nwdl, &nwdc);
            float *pa = nullptr, *pdl = nullptr, *pdc = nullptr;
            if (dmalloc(d, &pa, nwa) || dmalloc(d, &pdl, nwdl) || dmalloc(d, &pdc, nwdc) ||
                dmalloc(d, &d->rw.wf, (size_t)nfused * (HDEC + ENC)) || dmalloc(d, &d->rw.bf, nfused) ||
                dmalloc(d, &d->rw.ba, RES_CUS * 16) || dmalloc(d, &d->rw.bd, RES_CUS * 16) ||
                dmalloc(d, &d->rw.w2, (size_t)PRE * PRE) || dmalloc(d, &d->rw.b2, PRE) ||
                dmalloc(d, &d->rw.wq, (size_t)ADIM * HATT) ||
                dmalloc(d, &d->gran, (size_t)2 * GR_TOTAL + 2))
                e = hipErrorOutOfMemory;
            if (e == hipSuccess) {
                d->rw.wa = reinterpret_cast<float4*>(pa);
                d->rw.wdl = reinterpret_cast<float4*>(pdl);
                d->rw.wdc = reinterpret_cast<float4*>(pdc);
                ResSrc src{a_wih, a_whh, a_bih, a_bhh, d_wih, d_whh, d_bih, d_bhh, w_p1, d->b_pre2, wq, wf, bf, nfused};
                e = resident_pack(src, d->rw, s);
                // small batches: the batched resident decoder (both LSTMs' rows in registers) for the
                // attention configurations it covers; TTS_RESIDENT_BATCH=0 keeps them multi-launch
                const int gen = GEN_ON | (cfg->attn_norm == 0 ? GEN_SOFTMAX : 0) | (cfg->forward_attn ? GEN_FORWARD : 0) |
                                (cfg->forward_attn && cfg->forward_attn_mask ? GEN_MASK : 0) |
                                (cfg->forward_attn && cfg->trans_agent ? GEN_TA : 0) | (cfg->location_attn ? GEN_LOCATION : 0) |
                                (cfg->windowing ? GEN_WINDOW : 0);
                const char* rbe = getenv("TTS_RESIDENT_BATCH");
                if (e == hipSuccess && cfg->max_batch >= 2 && resident_batch_supports(gen) && !(rbe && rbe[0] == '0') &&
                    resident_batch_prepare() == hipSuccess) {
                    size_t nra, nrd;
                    resident_batch_weight_floats(&nra, &nrd);
                    float *qa = nullptr, *qd = nullptr;
                    if (dmalloc(d, &qa, nra) || dmalloc(d, &qd, nrd) || dmalloc(d, &d->rb_gran, resident_batch_granules() + 2))
                        e = hipErrorOutOfMemory;
                    if (e == hipSuccess) {
                        d->rb_wa = reinterpret_cast<float4*>(qa);
                        d->rb_wd = reinterpret_cast<float4*>(qd);
                        e = resident_batch_pack(src, d->rb_wa, d->rb_wd, s);
                        if (e == hipSuccess)
                            e = hipMemsetAsync(d->rb_gran, 0, sizeof(unsigned long long) * (resident_batch_granules() + 2), s);
                    }
                    if (e == hipSuccess) {
                        d->rbatch = true;
                        d->rb_gen = gen;
                    }
                }
            }
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        (void)hipFree(wf);
        (void)hipFree(bf);
        HK(e);
    }
    // small weights in reference layout
    CK(copy_weight(d, &d->v, vw, ADIM, s));
    CK(copy_weight(d, &d->v_b, vb, 1, s));
    CK(copy_weight(d, &d->W_in, win, (size_t)ADIM * ENC, s));
    CK(copy_weight(d, &d->att_init, ainit, HATT, s));
    CK(copy_weight(d, &d->dec_init, dinit, HDEC, s));
    CK(copy_weight(d, &d->go, goinit, nmel, s));
    if (taw) {
        CK(copy_weight(d, &d->ta_w, taw, HATT + ENC, s));
        CK(copy_weight(d, &d->ta_b, tab, 1, s));
    }
    if (lcw) {
        CK(copy_weight(d, &d->loc_conv, lcw, NLOC * 2 * KLOC, s));
        CK(copy_weight(d, &d->loc_dense, ldw, ADIM * NLOC, s));
        if (d->resident && d->res_gen) {
            CK(dmalloc(d, &d->loc_conv_p, 2 * NLOC * 32));
            HK(resident_pack_location(d->loc_conv, d->loc_conv_p, s));
        }
    }
    // workspace
    const int Bc = cfg->max_batch, Lc = (cfg->max_len + 3) / 4 * 4;
    d->Bcap = Bc;
    d->Lcap = Lc;
    d->hist_cap = cfg->max_steps + 21;
    CK(dmalloc(d, &d->enc, (size_t)Bc * Lc * ENC));
    CK(dmalloc(d, &d->Pt, (size_t)Bc * ADIM * Lc));
    CK(dmalloc(d, &d->h_att, (size_t)2 * Bc * HATT));
    CK(dmalloc(d, &d->c_att, (size_t)Bc * HATT));
    CK(dmalloc(d, &d->h_dec, (size_t)2 * Bc * HDEC));
    CK(dmalloc(d, &d->c_dec, (size_t)Bc * HDEC));
    CK(dmalloc(d, &d->xa, (size_t)2 * Bc * XA));
    CK(dmalloc(d, &d->mem, (size_t)Bc * nmel));
    CK(dmalloc(d, &d->pre1, (size_t)Bc * PRE));
    CK(dmalloc(d, &d->pre1_go, (size_t)PRE));
    CK(dmalloc(d, &d->q, (size_t)Bc * ADIM));
    if (Bc > 16) {
        d->ntf = (Bc + 15) / 16;
        const size_t rows = (size_t)d->ntf * 16;
        CK(dmalloc(d, &d->xaf, 2 * rows * XA));
        CK(dmalloc(d, &d->hattf, 2 * rows * HATT));
        CK(dmalloc(d, &d->hdecf, 2 * rows * HDEC));
        CK(dmalloc(d, &d->pre1f, rows * PRE));
    }
    CK(dmalloc(d, &d->epart, (size_t)Bc * QE_TILES * Lc));
    if (cfg->location_attn) CK(dmalloc(d, &d->locf, (size_t)Bc * NLOC * Lc));
    // alpha / att_cum / win_idx / nidx: two parity slots (the split general attention launch reads
    // slot t & 1 and writes the other; the fast paths use slot 0 only)
    CK(dmalloc(d, &d->alpha, (size_t)2 * Bc * Lc));
    CK(dmalloc(d, &d->att_w, (size_t)Bc * Lc));
    CK(dmalloc(d, &d->att_cum, (size_t)2 * Bc * Lc));
    CK(dmalloc(d, &d->u, Bc));
    CK(dmalloc(d, &d->tail, Bc));
    CK(dmalloc(d, &d->lens, Bc));
    CK(dmalloc(d, &d->win_idx, 2 * Bc));
    CK(dmalloc(d, &d->nidx, 2 * Bc));
    CK(dmalloc(d, &d->flag1, Bc));
    CK(dmalloc(d, &d->count, Bc));
    CK(dmalloc(d, &d->done, Bc));
    CK(dmalloc(d, &d->n_steps, Bc));
    CK(dmalloc(d, &d->state, 8));  // {step, n_active} x 2 parities (kernels load one slot as int2), stop_acc
    CK(dmalloc(d, &d->mel_hist, (size_t)Bc * d->hist_cap * nmel));
    CK(dmalloc(d, &d->stop_hist, (size_t)Bc * d->hist_cap));
    CK(dmalloc(d, &d->align_hist, (size_t)Bc * d->hist_cap * Lc));
    HK(attention_prepare(Lc, cfg->location_attn));
    HK(hipMemsetAsync(d->xa, 0, sizeof(float) * 2 * Bc * XA, s));
    HK(hipMemsetAsync(d->h_att, 0, sizeof(float) * 2 * Bc * HATT, s));
    HK(hipMemsetAsync(d->h_dec, 0, sizeof(float) * 2 * Bc * HDEC, s));
    HK(hipMemsetAsync(d->mem, 0, sizeof(float) * Bc * nmel, s));
    HK(hipMemsetAsync(d->enc, 0, sizeof(float) * Bc * Lc * ENC, s));
    HK(hipMemsetAsync(d->Pt, 0, sizeof(float) * Bc * ADIM * Lc, s));
    HK(hipMemsetAsync(d->state, 0, sizeof(int) * 8, s));
    HK(hipStreamSynchronize(s));
#undef CK
#undef HK
    *out = d;
    return TTS_OK;
}

void tts_decoder_destroy(tts_decoder* d) {
    if (!d) return;
    if (d->stream) (void)hipStreamSynchronize(d->stream);
    for (auto& kv : d->graphs) {
        for (auto* x : {kv.second.step[0], kv.second.step[1], kv.second.chunk})
            if (x) (void)hipGraphExecDestroy(x);
    }
    for (void* p : d->allocs) (void)hipFree(p);
    if (d->host_flags) (void)hipHostFree(d->host_flags);
    for (hipEvent_t e : {d->ev_in, d->ev_out, d->ev_t0, d->ev_t1, d->ev_sync})
        if (e) (void)hipEventDestroy(e);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    delete d;
}

tts_status tts_decoder_run(tts_decoder* d, const float* enc, const int32_t* lens, int B, int Lmax, int max_steps,
                           int steps_cap, float* mel, float* stop, float* align, int32_t* n_steps, void* stream) {
    return decoder_run(d, enc, lens, B, Lmax, max_steps, steps_cap, mel, stop, align, n_steps, stream, false);
}

tts_status tts_decoder_run_teacher(tts_decoder* d, const float* enc, const int32_t* lens, int B, int Lmax,
                                   const float* memories, int64_t mem_ldb, int steps, float* mel, float* stop,
                                   float* align, void* stream) {
    TTS_CHECK(d && enc && lens && memories && mel && stop, TTS_ERR_INVALID, "null argument");
    TTS_CHECK(B >= 1 && B <= d->Bcap, TTS_ERR_INVALID, "batch exceeds decoder capacity");
    TTS_CHECK(Lmax >= 2 && Lmax <= d->Lcap, TTS_ERR_INVALID, "Lmax exceeds decoder capacity");
    TTS_CHECK(steps >= 1 && steps <= d->hist_cap, TTS_ERR_INVALID, "teacher steps exceed the decoder's history capacity");
    TTS_CHECK(mem_ldb >= (int64_t)(steps - 1) * d->nmel, TTS_ERR_INVALID, "teacher memory rows too short");
    for (int b = 0; b < B; ++b)
        TTS_CHECK(lens[b] >= 2 && lens[b] <= Lmax, TTS_ERR_INVALID, "encoder length out of range [2, Lmax]");
    hipStream_t cs = static_cast<hipStream_t>(stream);
    hipStream_t s = d->stream;
    TTS_HIP(hipEventRecord(d->ev_in, cs));
    TTS_HIP(hipStreamWaitEvent(s, d->ev_in, 0));
    TTS_HIP(hipMemcpy2DAsync(d->enc, (size_t)d->Lcap * ENC * 4, enc, (size_t)Lmax * ENC * 4, (size_t)Lmax * ENC * 4, B,
                             hipMemcpyDeviceToDevice, s));
    TTS_HIP(hipMemcpyAsync(d->lens, lens, sizeof(int) * B, hipMemcpyHostToDevice, s));
    TTS_HIP(launch_project_inputs(d->enc, d->W_in, B, Lmax, d->Lcap, d->Pt, s));
    InitArgs ia{};
    ia.B = B; ia.Lcap = d->Lcap; ia.nmel = d->nmel; ia.lens = d->lens;
    ia.att_init = d->att_init; ia.dec_init = d->dec_init; ia.go = d->go;
    ia.h_att = d->h_att; ia.h_pstride = (int64_t)d->Bcap * HATT; ia.c_att = d->c_att;
    ia.h_dec = d->h_dec; ia.c_dec = d->c_dec; ia.xa = d->xa; ia.xa_pstride = (int64_t)d->Bcap * XA; ia.mem = d->mem;
    ia.alpha = d->alpha; ia.att_w = d->att_w; ia.att_cum = d->att_cum; ia.u = d->u; ia.win_idx = d->win_idx;
    ia.locf = d->locf;
    ia.nidx = d->nidx; ia.tail = d->tail; ia.flag1 = d->flag1; ia.count = d->count; ia.done = d->done; ia.n_steps = d->n_steps;
    ia.step = d->state; ia.n_active = d->state + 1;
    TTS_HIP(launch_decoder_init(ia, s));
    if (frag_on(d, B)) { tts_status fs = enqueue_frag_sync(d, B, s); if (fs) return fs; }
    // step t: memory = go frame (t = 0) or teacher row t-1 -> prenet layer 1 (reference weights, no
    // fold) -> the inference step with the stop rule off (its fused launch's prenet-1 output is
    // overwritten by the next step's teacher frame)
    for (int t = 0; t < steps; ++t) {
        const int p = t & 1;
        TTS_HIP(launch_teacher_memory(memories, mem_ldb, d->nmel, d->state + 2 * p, d->mem, B, s));
        tts_status st = enqueue_prenet_go(d, B, s, d->state + 2 * p);
        if (!st) st = enqueue_step(d, B, Lmax, steps, p, s, nullptr, 2);
        if (st) return st;
    }
    const size_t nm = d->nmel;
    TTS_HIP(hipMemcpy2DAsync(mel, (size_t)steps * nm * 4, d->mel_hist, (size_t)d->hist_cap * nm * 4, (size_t)steps * nm * 4,
                             B, hipMemcpyDeviceToDevice, s));
    TTS_HIP(hipMemcpy2DAsync(stop, (size_t)steps * 4, d->stop_hist, (size_t)d->hist_cap * 4, (size_t)steps * 4, B,
                             hipMemcpyDeviceToDevice, s));
    if (align)
        TTS_HIP(hipMemcpy2DAsync(align, (size_t)steps * Lmax * 4, d->align_hist, (size_t)d->hist_cap * Lmax * 4,
                                 (size_t)steps * Lmax * 4, B, hipMemcpyDeviceToDevice, s));
    TTS_HIP(hipEventRecord(d->ev_out, s));
    TTS_HIP(hipStreamWaitEvent(cs, d->ev_out, 0));
    d->last_resident = 0;
    d->last_steps_done = 0;  // a later run_continue must start from a regular run
    return TTS_OK;
}

tts_status tts_decoder_run_continue(tts_decoder* d, const float* enc, const int32_t* lens, int B, int Lmax,
                                    int max_steps, int steps_cap, float* mel, float* stop, float* align,
                                    int32_t* n_steps, void* stream) {
    TTS_CHECK(d && B == 1, TTS_ERR_UNSUPPORTED, "continuous (truncated) decoding is batch-1, as the reference's");
    TTS_CHECK(d->last_B == 1 && d->last_steps_done > 0, TTS_ERR_INVALID,
              "tts_decoder_run_continue needs a previous batch-1 tts_decoder_run / _continue");
    return decoder_run(d, enc, lens, B, Lmax, max_steps, steps_cap, mel, stop, align, n_steps, stream, true);
}

}  // extern "C"

namespace {
tts_status decoder_run(tts_decoder* d, const float* enc, const int32_t* lens, int B, int Lmax, int max_steps,
                       int steps_cap, float* mel, float* stop, float* align, int32_t* n_steps, void* stream, bool keep) {
    TTS_CHECK(d && enc && lens && mel && stop && n_steps, TTS_ERR_INVALID, "null argument");
    TTS_CHECK(B >= 1 && B <= d->Bcap, TTS_ERR_INVALID, "batch exceeds decoder capacity");
    TTS_CHECK(Lmax >= 2 && Lmax <= d->Lcap, TTS_ERR_INVALID, "Lmax exceeds decoder capacity");
    TTS_CHECK(max_steps >= 1 && max_steps <= d->cfg.max_steps, TTS_ERR_INVALID, "max_steps exceeds decoder capacity");
    TTS_CHECK(steps_cap >= max_steps + 20, TTS_ERR_INVALID, "steps_cap must be >= max_steps + 20");
    int first = 0;
    for (int b = 0; b < B; ++b) {
        TTS_CHECK(lens[b] >= 2 && lens[b] <= Lmax, TTS_ERR_INVALID, "encoder length out of range [2, Lmax]");
        first = std::max(first, std::min(2 * lens[b] + 22, max_steps));
    }
    hipStream_t cs = static_cast<hipStream_t>(stream);
    hipStream_t s = d->pipeline ? cs : d->stream;
    if (s != cs) {
        TTS_HIP(hipEventRecord(d->ev_in, cs));
        TTS_HIP(hipStreamWaitEvent(s, d->ev_in, 0));
    }
    // A fresh batch-1 resident run ("direct") reads the caller's encoder output in place, the length
    // from the pipeline's device array when it has one, zeroes its hand-off granules and takes the
    // cached go-frame prenet row inside decoder_init: two launches before the resident one instead
    // of six.  A fallback to the multi-launch path stages the copies first (stage_fallback).
    const bool direct = d->resident && B == 1 && lens[0] <= RES_LMAX && !keep;
    if (!direct)
        TTS_HIP(hipMemcpy2DAsync(d->enc, (size_t)d->Lcap * ENC * 4, enc, (size_t)Lmax * ENC * 4, (size_t)Lmax * ENC * 4,
                                 B, hipMemcpyDeviceToDevice, s));
    const int* lens_dev = direct && d->io_lens ? d->io_lens : d->lens;
    if (lens_dev == d->lens) TTS_HIP(hipMemcpyAsync(d->lens, lens, sizeof(int) * B, hipMemcpyHostToDevice, s));
    // (the memory projection goes out with the init launch below, unless the VALU form is asked for)
    static const bool proj_valu = [] {  // measurement: TTS_PROJ_VALU=1, the VALU projection launch
        const char* v = getenv("TTS_PROJ_VALU");
        return v && v[0] == '1';
    }();
    const bool proj_fused = !proj_valu;
    if (!proj_fused) TTS_HIP(launch_project_inputs(direct ? enc : d->enc, d->W_in, B, Lmax, d->Lcap, d->Pt, s));
    d->last_enc_direct = direct ? enc : nullptr;
    d->last_len_direct = lens[0];
    InitArgs ia{};
    ia.B = B; ia.Lcap = d->Lcap; ia.nmel = d->nmel; ia.lens = lens_dev;
    ia.att_init = d->att_init; ia.dec_init = d->dec_init; ia.go = d->go;
    ia.h_att = d->h_att; ia.h_pstride = (int64_t)d->Bcap * HATT; ia.c_att = d->c_att;
    ia.h_dec = d->h_dec; ia.c_dec = d->c_dec; ia.xa = d->xa; ia.xa_pstride = (int64_t)d->Bcap * XA; ia.mem = d->mem;
    ia.alpha = d->alpha; ia.att_w = d->att_w; ia.att_cum = d->att_cum; ia.u = d->u; ia.win_idx = d->win_idx;
    ia.locf = d->locf;
    ia.nidx = d->nidx; ia.tail = d->tail; ia.flag1 = d->flag1; ia.count = d->count; ia.done = d->done; ia.n_steps = d->n_steps;
    ia.step = d->state; ia.n_active = d->state + 1;
    if (keep) {
        // Decoder.inference_truncated (layers/tacotron2.py:287-328): attention / stop state restart,
        // the RNN states, context and memory (the last mel frame) carry over.  The last step of the
        // previous run (parity (n-1) & 1) left h_att / h_dec in its slot, the context in the other
        // parity's xa row, and relu(W1 mel_last) in pre1 (the fused mel launch computes the next
        // step's prenet layer 1): move them to the slots step 0 reads.
        const int pl = (d->last_steps_done - 1) & 1;
        const size_t hp = (size_t)d->Bcap * HATT;
        if (pl != 1) {
            TTS_HIP(hipMemcpyAsync(d->h_att + hp, d->h_att, HATT * sizeof(float), hipMemcpyDeviceToDevice, s));
            TTS_HIP(hipMemcpyAsync(d->h_dec + hp, d->h_dec, HDEC * sizeof(float), hipMemcpyDeviceToDevice, s));
        }
        if (1 - pl != 0)
            TTS_HIP(hipMemcpyAsync(d->xa + PRE, d->xa + (size_t)d->Bcap * XA + PRE, ENC * sizeof(float),
                                   hipMemcpyDeviceToDevice, s));
        ia.keep = 1;
    }
    if (direct) {
        ia.zero = d->gran;
        ia.nzero = 2 * GR_TOTAL + 2;
        ia.pre1 = d->pre1;
        ia.pre1_go = d->pre1_go_ok ? d->pre1_go : nullptr;
    }
    if (proj_fused) TTS_HIP(launch_project_init(direct ? enc : d->enc, d->W_in, B, Lmax, d->Lcap, d->Pt, ia, s));
    else TTS_HIP(launch_decoder_init(ia, s));
    if (frag_on(d, B)) { tts_status fs = enqueue_frag_sync(d, B, s); if (fs) return fs; }
    if (!keep && !ia.pre1_go) {
        tts_status st = enqueue_prenet_go(d, B, s);
        if (st) return st;
        if (direct) {
            TTS_HIP(hipMemcpyAsync(d->pre1_go, d->pre1, PRE * sizeof(float), hipMemcpyDeviceToDevice, s));
            d->pre1_go_ok = true;
        }
    }
    // a direct run falling back to the multi-launch path: the staged inputs the step graphs read
    auto stage_fallback = [&]() -> tts_status {
        if (!direct) return TTS_OK;
        TTS_HIP(hipMemcpy2DAsync(d->enc, (size_t)d->Lcap * ENC * 4, enc, (size_t)Lmax * ENC * 4, (size_t)Lmax * ENC * 4,
                                 B, hipMemcpyDeviceToDevice, s));
        if (ia.lens != d->lens) TTS_HIP(hipMemcpyAsync(d->lens, lens, sizeof(int) * B, hipMemcpyHostToDevice, s));
        ia.lens = d->lens;
        ia.zero = nullptr;
        ia.nzero = 0;
        ia.pre1_go = nullptr;
        d->last_enc_direct = nullptr;
        return TTS_OK;
    };
    int run = 0;  // steps enqueued; the next step has parity run & 1
    d->last_resident = 0;
    // stage timers (tts_decoder_last_timing) outside pipeline mode only: every event marker holds
    // the GPU ~5.8 us between the kernels around it
    const bool timed = !d->pipeline;
    bool res_done = false;
    static const bool verbose = [] {
        const char* v = getenv("TTS_VERBOSE");
        return v && v[0] == '1';
    }();
    if (verbose)
        fprintf(stderr, "[tts] decoder_run B=%d L=%d resident=%d gen=%d keep=%d direct=%d\n", B, lens[0],
                (int)d->resident, d->res_gen, (int)keep, (int)direct);
    // consecutive launches of <= RB_MAXB sentences beat the multi-launch step (~45 us at any batch up
    // to 64) only for a few groups: TTS_RB_MAX (default rb_max_batch()) bounds the batch
    bool rb_ok = d->rbatch && B >= 2 && B <= rb_max_batch() && !keep;
    static const bool rb_prof = [] {
        const char* v = getenv("TTS_RB_PROF");
        return v && v[0] == '1';
    }();
    for (int b = 0; rb_ok && b < B; ++b) rb_ok = lens[b] <= RES_LMAX;
    if (rb_ok) {
        // batches: one persistent launch per group of <= RB_MAXB sentences (resident_batch.hip),
        // each sentence's state, histories and step count in the multi-launch path's slots
        if (timed) TTS_HIP(hipEventRecord(d->ev_t0, s));
        bool all = true;
        for (int g0 = 0; g0 < B && all; g0 += RB_MAXB) {
            const int nb = std::min(RB_MAXB, B - g0);
            ResBatchArgs rb{};
            rb.B = nb;
            rb.gen = d->rb_gen;
            for (int b = 0; b < nb; ++b) rb.L[b] = lens[g0 + b];
            rb.Lcap = d->Lcap; rb.nmel = d->nmel; rb.nrows = d->nmel + PRE + 1; rb.max_steps = max_steps;
            rb.hist_cap = d->hist_cap; rb.Lalign = Lmax; rb.timeout_ticks = d->res_ticks;
            rb.wa = d->rb_wa; rb.wd = d->rb_wd;
            rb.w2 = d->rw.w2; rb.b2 = d->rw.b2; rb.wq = d->rw.wq; rb.wf = d->rw.wf; rb.bf = d->rw.bf; rb.ba = d->rw.ba;
            rb.bd = d->rw.bd;
            rb.v = d->v; rb.v_b = d->v_b;
            rb.Pt = d->Pt + (size_t)g0 * ADIM * d->Lcap;
            rb.enc = d->enc + (size_t)g0 * d->Lcap * ENC;
            rb.h_att = d->h_att + (size_t)g0 * HATT; rb.c_att = d->c_att + (size_t)g0 * HATT;
            rb.h_dec = d->h_dec + (size_t)g0 * HDEC; rb.c_dec = d->c_dec + (size_t)g0 * HDEC;
            rb.xa = d->xa + (size_t)g0 * XA;
            rb.hps = (int64_t)d->Bcap * HATT; rb.xps = (int64_t)d->Bcap * XA;
            rb.pre1 = d->pre1 + (size_t)g0 * PRE;
            rb.alpha = d->alpha + (size_t)g0 * d->Lcap;
            rb.nidx = d->nidx + g0; rb.u = d->u + g0; rb.flag1 = d->flag1 + g0; rb.count = d->count + g0;
            rb.done = d->done + g0; rb.n_steps = d->n_steps + g0;
            rb.mel_hist = d->mel_hist + (size_t)g0 * d->hist_cap * d->nmel;
            rb.stop_hist = d->stop_hist + (size_t)g0 * d->hist_cap;
            rb.align_hist = d->align_hist + (size_t)g0 * d->hist_cap * Lmax;
            rb.gran = d->rb_gran;
            auto knob = [](const char* name, int dflt) {
                const char* v = getenv(name);
                return v ? atoi(v) : dflt;
            };
            static const int rb_hatt = knob("TTS_RB_SLEEP_HATT", 0), rb_hdec = knob("TTS_RB_SLEEP_HDEC", 0),
                             rb_pre2 = knob("TTS_RB_SLEEP_PRE2", 0), rb_ctx = knob("TTS_RB_SLEEP_CTX", 0);
            rb.sleep_hatt = rb_hatt;
            rb.sleep_hdec = rb_hdec;
            rb.sleep_pre2 = rb_pre2;
            rb.sleep_ctx = rb_ctx;
            rb.status = reinterpret_cast<int*>(d->rb_gran + resident_batch_granules());
            if (rb_prof && !d->rb_prof) {
                tts_status ps = dmalloc(d, &d->rb_prof, (size_t)RES_CUS * 4 * RB_PROF_SLOTS);
                if (ps) return ps;
            }
            rb.prof = rb_prof ? d->rb_prof : nullptr;
            bool wrapped = false;
            d->rb_salt = res_next_salt(d->rb_salt, &wrapped);
            rb.salt = d->rb_salt;
            if (wrapped)
                TTS_HIP(hipMemsetAsync(d->rb_gran, 0, sizeof(unsigned long long) * (resident_batch_granules() + 2), s));
            TTS_HIP(hipMemsetAsync(rb.status, 0, 4 * sizeof(int), s));
            bool launched = false;
            TTS_HIP(launch_resident_batch(rb, s, &launched));
            if (verbose) fprintf(stderr, "[tts] resident batch launch g0=%d nb=%d launched=%d\n", g0, nb, (int)launched);
            if (!launched) {
                d->rbatch = false;  // the grid cannot be co-resident on this device
                all = false;
                break;
            }
            TTS_HIP(hipMemcpyAsync(d->host_flags, rb.status, sizeof(int), hipMemcpyDeviceToHost, s));
            TTS_HIP(hipMemcpyAsync(d->host_flags + 4 + g0, d->n_steps + g0, sizeof(int) * nb, hipMemcpyDeviceToHost, s));
            TTS_HIP(spin_sync(s, d->ev_sync));
            if (verbose) fprintf(stderr, "[tts] resident batch status=%d\n", d->host_flags[0]);
            if (d->host_flags[0] != 0) {
                TTS_CHECK(d->host_flags[0] != 100, TTS_ERR_HIP, "decoder did not stop within max_steps + 20 (internal error)");
                if (d->host_flags[0] == RES_STATUS_PLACEMENT) {
                    if (++d->rb_place_fails >= RES_PLACEMENT_RETRIES) d->rbatch = false;
                } else {
                    ++d->res_timeouts;
                }
                all = false;
                break;
            }
            d->rb_place_fails = 0;
            if (rb_prof) {
                // TTS_RB_PROF=1: microseconds per step of each phase (wall clock 100 MHz) for every wave
                // index: min / mean / max over the 256 CUs, and CU 0
                std::vector<long long> pk((size_t)RES_CUS * 4 * RB_PROF_SLOTS);
                TTS_HIP(hipMemcpy(pk.data(), rb.prof, pk.size() * sizeof(long long), hipMemcpyDeviceToHost));
                const double steps = pk[RB_PROF_SLOTS - 1] > 0 ? (double)pk[RB_PROF_SLOTS - 1] : 1.0;
                fprintf(stderr, "[tts] resident batch nb=%d steps=%lld (us/step per phase: min/mean/max over CUs)\n", nb,
                        pk[RB_PROF_SLOTS - 1]);
                for (int w = 0; w < 4; ++w) {
                    fprintf(stderr, "[tts]  wave %d:", w);
                    for (int k : {0, 1, 2, 3, 4, 5, 6, 20, 21, 22, 23, 7, 8, 9, 10, 11, 12}) {
                        double mn = 1e30, mx = 0, sum = 0;
                        for (int cu = 0; cu < RES_CUS; ++cu) {
                            const double v = pk[((size_t)cu * 4 + w) * RB_PROF_SLOTS + k] * 0.01 / steps;
                            mn = std::min(mn, v);
                            mx = std::max(mx, v);
                            sum += v;
                        }
                        fprintf(stderr, " %d:%.2f/%.2f/%.2f", k, mn, sum / RES_CUS, mx);
                    }
                    fprintf(stderr, "\n");
                }
                // one step (RB_PROF_T): the last publisher of an edge vs each CU's arrival (us)
                if (pk[RB_PROF_SLOTS - 1] > RB_PROF_T) {
                    auto at = [&](int cu, int w, int k) { return pk[((size_t)cu * 4 + w) * RB_PROF_SLOTS + k]; };
                    const char* names[] = {"h_att", "h_dec"};
                    const int pubk[] = {13, 16}, donek[] = {14, 17};
                    for (int e = 0; e < 2; ++e) {
                        long long pmin = LLONG_MAX, pmax = 0, dmin = LLONG_MAX, dmax = 0;
                        int pmax_cu = -1;
                        for (int cu = 0; cu < RES_CUS; ++cu)
                            for (int w = 0; w < 4; ++w) {
                                const long long p = at(cu, w, pubk[e]), q = at(cu, w, donek[e]);
                                if (p < pmin) pmin = p;
                                if (p > pmax) { pmax = p; pmax_cu = cu * 4 + w; }
                                dmin = std::min(dmin, q);
                                dmax = std::max(dmax, q);
                            }
                        fprintf(stderr, "[tts]  step %d %s: publish spread %.2f us (last: CU %d wave %d), arrival after the last publish %.2f .. %.2f us\n",
                                RB_PROF_T, names[e], (pmax - pmin) * 0.01, pmax_cu / 4, pmax_cu % 4, (dmin - pmax) * 0.01,
                                (dmax - pmax) * 0.01);
                    }
                }
            }
        }
        if (all) {
            if (timed) TTS_HIP(hipEventRecord(d->ev_t1, s));
            std::copy(d->host_flags + 4, d->host_flags + 4 + B, n_steps);
            run = 0;
            for (int b = 0; b < B; ++b) run = std::max(run, (int)n_steps[b]);
            res_done = true;
            d->last_resident = 2;
        } else {
            // re-run the whole batch on the multi-launch path from its initial state
            TTS_HIP(launch_decoder_init(ia, s));
            if (frag_on(d, B)) { tts_status fs = enqueue_frag_sync(d, B, s); if (fs) return fs; }
            tts_status st = enqueue_prenet_go(d, B, s);
            if (st) return st;
        }
    }
    if (!res_done && d->resident && B == 1 && lens[0] <= RES_LMAX) {
        // one persistent launch runs every step (resident.h); same state / history buffers
        ResArgs ra{};
        ra.w = d->rw;
        ra.L = lens[0]; ra.Lcap = d->Lcap; ra.nmel = d->nmel; ra.nrows = d->nmel + PRE + 1;
        ra.max_steps = max_steps; ra.hist_cap = d->hist_cap; ra.Lalign = Lmax; ra.timeout_ticks = d->res_ticks;
        ra.v = d->v; ra.v_b = d->v_b; ra.Pt = d->Pt; ra.enc = direct ? enc : d->enc;
        ra.h_att = d->h_att; ra.c_att = d->c_att; ra.h_dec = d->h_dec; ra.c_dec = d->c_dec; ra.xa = d->xa;
        ra.hps = (int64_t)d->Bcap * HATT; ra.xps = (int64_t)d->Bcap * XA;
        ra.pre1 = d->pre1; ra.alpha = d->alpha; ra.nidx = d->nidx; ra.u = d->u; ra.flag1 = d->flag1; ra.count = d->count;
        ra.done = d->done; ra.n_steps = d->n_steps;
        ra.mel_hist = d->mel_hist; ra.stop_hist = d->stop_hist; ra.align_hist = d->align_hist;
        ra.gen = d->res_gen;
        ra.ta_w = d->ta_w; ra.ta_b = d->ta_b; ra.att_w0 = d->att_w; ra.att_cum0 = d->att_cum; ra.win0 = d->win_idx;
        ra.loc_conv = d->loc_conv_p; ra.loc_dense = d->loc_dense;
        ra.gran = d->gran;
        // first-poll delays (resident.h; round 6: h_att 5 / h_dec 5 took a configs[1] sentence from
        // 2.65 to 2.29 ms, tools/cases_sleep.txt); TTS_RES_SLEEP_* override them
        auto knob = [](const char* name, int dflt) {
            const char* v = getenv(name);
            return v ? atoi(v) : dflt;
        };
        static const int sl_hatt = knob("TTS_RES_SLEEP_HATT", 5), sl_hdec = knob("TTS_RES_SLEEP_HDEC", 5),
                         sl_p1 = knob("TTS_RES_SLEEP_P1", 0), sl_pre2 = knob("TTS_RES_SLEEP_PRE2", 2),
                         sl_ctx = knob("TTS_RES_SLEEP_CTX", 0), sl_q = knob("TTS_RES_SLEEP_Q", 0),
                         sl_e = knob("TTS_RES_SLEEP_E", 0);
        ra.sleep_hatt = sl_hatt;
        ra.sleep_hdec = sl_hdec;
        ra.sleep_p1 = sl_p1;
        ra.sleep_pre2 = sl_pre2;
        ra.sleep_ctx = sl_ctx;
        ra.sleep_q = sl_q;
        ra.sleep_e = sl_e;
        ra.status = reinterpret_cast<int*>(d->gran + 2 * GR_TOTAL);
        // direct (pipelined) runs skip the per-launch clear and rely on the 18-bit tag salt: on a
        // salt wrap a granule left 2^18 launches back could match a current wait, so clear then
        bool wrapped = false;
        d->res_salt = res_next_salt(d->res_salt, &wrapped);
        ra.salt = d->res_salt;
        d->last_ra = ra;
        if (!direct || wrapped)
            TTS_HIP(hipMemsetAsync(d->gran, 0, sizeof(unsigned long long) * (2 * GR_TOTAL + 2), s));
        if (timed) TTS_HIP(hipEventRecord(d->ev_t0, s));
        bool launched = false;
        TTS_HIP(launch_resident(ra, s, &launched));
        if (verbose) fprintf(stderr, "[tts] resident launch: launched=%d\n", (int)launched);
        if (!launched) {
            // the grid cannot be co-resident on this device (launch_persistent): nothing ran and the
            // initial state is untouched; the multi-launch path takes over for the life of the handle
            d->resident = false;
            if (tts_status st = stage_fallback()) return st;
            TTS_HIP(launch_decoder_init(ia, s));
            if (!keep) { tts_status st = enqueue_prenet_go(d, B, s); if (st) return st; }
        } else {
        if (timed) TTS_HIP(hipEventRecord(d->ev_t1, s));
        const int seq = ++d->rb_seq;
        {
            // status, step counts (and the pipeline's extra word / GL clamp) in one launch, then the
            // sequence word the host polls
            Readback rb{};
            rb.src[0] = ra.status; rb.n[0] = 1; rb.dst[0] = d->host_flags;
            rb.src[1] = d->n_steps; rb.n[1] = B; rb.dst[1] = d->host_flags + 4;
            rb.count = 2;
            if (d->io_rb_src) { rb.src[2] = d->io_rb_src; rb.n[2] = 1; rb.dst[2] = d->io_rb_dst; rb.count = 3; }
            if (d->io_clamp) {
                rb.clamp_src = d->n_steps; rb.clamp_dst = d->io_clamp; rb.clamp_n = B; rb.clamp_max = d->io_clamp_max;
            }
            rb.seq_dst = d->host_flags + 3;
            rb.seq = seq;
            TTS_HIP(readback(rb, s));
        }
        // a polling wait on the read-back's sequence word (no event marker); work that needs no
        // host-side step count (the synthesis postnet, Griffin-Lim) is enqueued before it, so the
        // device does not idle while the host wakes
        if (d->post_hook) {
            d->post_hook(d->post_ctx, s);
            d->hook_ran = true;
        }
        TTS_HIP(spin_word(d->host_flags + 3, seq, s));
        n_steps[0] = d->host_flags[4];
        if (verbose) fprintf(stderr, "[tts] resident status=%d steps=%d\n", d->host_flags[0], n_steps[0]);
        if (d->host_flags[0] == RES_STATUS_PLACEMENT) {
            // the runtime placed fewer than RES_MIN_CUS_PER_XCD workgroups on some XCD (or, for the
            // general form, more than that on one): the kernel stopped before touching any state.
            // This sentence runs multi-launch; the handle gives the resident path up only after
            // RES_PLACEMENT_RETRIES such sentences in a row (one uneven dispatch is not a device that
            // cannot place the grid: ADVICE r5)
            if (++d->res_place_fails >= RES_PLACEMENT_RETRIES) d->resident = false;
            if (verbose)
                fprintf(stderr, "[tts] resident decoder: placement failed (%d in a row)%s\n", d->res_place_fails,
                        d->resident ? "" : ", multi-launch from now on");
            if (tts_status st = stage_fallback()) return st;
            TTS_HIP(launch_decoder_init(ia, s));
            if (!keep) { tts_status st = enqueue_prenet_go(d, B, s); if (st) return st; }
        } else if (d->host_flags[0] != 0 && d->host_flags[0] != 100 && !keep) {
            // a hand-off wait timed out (a workgroup could not become resident beside another
            // stream's work, e.g. a pipelined Griffin-Lim): every wave drained with the status and
            // the grid is gone.  Re-run this sentence from its initial state on the multi-launch
            // path (same results within the resident tests' tolerance); the handle stays resident.
            // (inference_truncated's carried state may already be overwritten: that case raises.)
            ++d->res_timeouts;
            if (verbose) {
                int dbg[3] = {0, 0, 0};
                (void)hipMemcpy(dbg, ra.status, sizeof(dbg), hipMemcpyDeviceToHost);
                fprintf(stderr, "[tts] resident decoder: wait %d timed out at step %d on workgroup %d (L=%d); "
                                "re-running multi-launch\n", dbg[0], dbg[1], dbg[2], lens[0]);
            }
            if (tts_status st = stage_fallback()) return st;
            TTS_HIP(launch_decoder_init(ia, s));
            if (frag_on(d, B)) { tts_status fs = enqueue_frag_sync(d, B, s); if (fs) return fs; }
            tts_status st = enqueue_prenet_go(d, B, s);
            if (st) return st;
        } else {
            TTS_CHECK(d->host_flags[0] == 0, TTS_ERR_HIP,
                      d->host_flags[0] == 100 ? "decoder did not stop within max_steps + 20 (internal error)"
                                              : "resident decoder: a hand-off wait timed out (internal error)");
            run = n_steps[0];
            res_done = true;
            d->last_resident = 1;
            d->res_place_fails = 0;
        }
        }
    }
    if (!res_done) {
    auto key = std::make_tuple(B, Lmax, max_steps);
    auto it = d->graphs.find(key);
    if (it == d->graphs.end()) {
        Graphs g;
        tts_status st = build_graph(d, B, Lmax, max_steps, 0, 1, &g.step[0]);
        if (!st) st = build_graph(d, B, Lmax, max_steps, 1, 1, &g.step[1]);
        if (!st) st = build_graph(d, B, Lmax, max_steps, 0, CHUNK, &g.chunk);
        if (st) return st;
        it = d->graphs.emplace(key, g).first;
    }
    const Graphs& g = it->second;
    if (timed) TTS_HIP(hipEventRecord(d->ev_t0, s));
    auto launch_steps = [&](int n) -> tts_status {
        while (n > 0) {
            if ((run & 1) == 0 && n >= CHUNK) {
                TTS_HIP(hipGraphLaunch(g.chunk, s));
                run += CHUNK;
                n -= CHUNK;
            } else {
                TTS_HIP(hipGraphLaunch(g.step[run & 1], s));
                ++run;
                --n;
            }
        }
        return TTS_OK;
    };
    tts_status st = launch_steps(first);
    if (st) return st;
    for (;;) {
        // n_active as seen by the next step (its parity slot)
        TTS_HIP(hipMemcpyAsync(d->host_flags, d->state + 2 * (run & 1), 2 * sizeof(int), hipMemcpyDeviceToHost, s));
        TTS_HIP(spin_sync(s, d->ev_sync));
        if (d->host_flags[1] == 0) break;
        TTS_CHECK(run < max_steps + 20, TTS_ERR_HIP, "decoder did not stop within max_steps + 20 (internal error)");
        st = launch_steps(CHUNK);
        if (st) return st;
    }
    if (timed) TTS_HIP(hipEventRecord(d->ev_t1, s));
    TTS_HIP(hipMemcpyAsync(d->host_flags + 4, d->n_steps, sizeof(int) * B, hipMemcpyDeviceToHost, s));
    if (d->io_rb_src) TTS_HIP(hipMemcpyAsync(d->io_rb_dst, d->io_rb_src, sizeof(int), hipMemcpyDeviceToHost, s));
    TTS_HIP(spin_sync(s, d->ev_sync));
    std::copy(d->host_flags + 4, d->host_flags + 4 + B, n_steps);
    }
    int nmax = 0;
    for (int b = 0; b < B; ++b) nmax = std::max(nmax, (int)n_steps[b]);
    const size_t nm = d->nmel;
    if (!d->keep_hist) {
    TTS_HIP(hipMemcpy2DAsync(mel, (size_t)steps_cap * nm * 4, d->mel_hist, (size_t)d->hist_cap * nm * 4,
                             (size_t)nmax * nm * 4, B, hipMemcpyDeviceToDevice, s));
    TTS_HIP(hipMemcpy2DAsync(stop, (size_t)steps_cap * 4, d->stop_hist, (size_t)d->hist_cap * 4, (size_t)nmax * 4, B,
                             hipMemcpyDeviceToDevice, s));
    if (align)
        TTS_HIP(hipMemcpy2DAsync(align, (size_t)steps_cap * Lmax * 4, d->align_hist, (size_t)d->hist_cap * Lmax * 4,
                                 (size_t)nmax * Lmax * 4, B, hipMemcpyDeviceToDevice, s));
    // the mel history is written unguarded by done[] (see EPI_MEL_FUSED): zero rows past n_steps
    TTS_HIP(launch_zero_tail(mel, (int64_t)steps_cap * nm, d->n_steps, (int)nm, nmax, B, s));
    }
    if (s != cs) {
        TTS_HIP(hipEventRecord(d->ev_out, s));
        TTS_HIP(hipStreamWaitEvent(cs, d->ev_out, 0));
    }
    d->last_ms = 0.f;  // (pipeline mode: not timed)
    if (timed) {
        // (the resident paths record ev_t1 after their last host sync: it may still be pending)
        TTS_HIP(hipEventSynchronize(d->ev_t1));
        TTS_HIP(hipEventElapsedTime(&d->last_ms, d->ev_t0, d->ev_t1));
    }
    d->last_steps = run;
    d->last_B = B;
    d->last_Lmax = Lmax;
    d->last_max_steps = max_steps;
    d->last_first = first;
    d->last_init = ia;
    d->last_init.keep = 0;
    d->last_steps_done = B == 1 ? (int)n_steps[0] : 0;
    return TTS_OK;
}
}  // namespace

namespace {
// Measurement only: re-run the last batch-1 resident sentence with timers (marks: per-phase tick
// sums of CU 0 and the logging attention CU; always: the per-CU event trace, kept in d->res_trace).
tts_status res_rerun(tts_decoder* d, bool marks, long long* h) {
    TTS_CHECK(d->last_resident == 1 && d->last_steps > 0, TTS_ERR_INVALID,
              "the resident decoder profile needs a previous resident tts_decoder_run");
    TTS_HIP(hipDeviceSynchronize());  // measurement only: nothing else (a pipeline GL) on the device
    hipStream_t s = d->stream;
    long long* prof = nullptr;
    TTS_HIP(hipMalloc(&prof, sizeof(long long) * RES_PROF_LL));
    TTS_HIP(hipMemsetAsync(prof, 0, sizeof(long long) * RES_PROF_LL, s));
    TTS_HIP(launch_decoder_init(d->last_init, s));
    tts_status st = enqueue_prenet_go(d, 1, s);
    ResArgs ra = d->last_ra;
    ra.prof = prof;
    ra.prof_marks = marks ? 1 : 0;
    if (!st) {
        TTS_HIP(hipMemsetAsync(d->gran, 0, sizeof(unsigned long long) * (2 * GR_TOTAL + 2), s));
        bool launched = false;
        TTS_HIP(launch_resident(ra, s, &launched));
        if (!launched) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(prof);
            TTS_CHECK(false, TTS_ERR_UNSUPPORTED, "resident decoder cannot be co-resident on this device now");
        }
    }
    TTS_HIP(hipMemcpyAsync(h, prof, sizeof(long long) * 2 * RES_PHASES, hipMemcpyDeviceToHost, s));
    d->res_trace.resize(RES_PROF_LL - 2 * RES_PHASES);
    TTS_HIP(hipMemcpyAsync(d->res_trace.data(), prof + 2 * RES_PHASES, sizeof(long long) * d->res_trace.size(),
                           hipMemcpyDeviceToHost, s));
    TTS_HIP(hipMemcpyAsync(d->host_flags, ra.status, sizeof(int), hipMemcpyDeviceToHost, s));
    TTS_HIP(hipStreamSynchronize(s));
    (void)hipFree(prof);
    if (st) return st;
    TTS_CHECK(d->host_flags[0] == 0, TTS_ERR_HIP, "resident decoder: a hand-off wait timed out (internal error)");
    return TTS_OK;
}
}  // namespace

extern "C" {

tts_status tts_decoder_last_timing(tts_decoder* d, float* loop_ms, int* steps_run) {
    TTS_CHECK(d && loop_ms && steps_run, TTS_ERR_INVALID, "null argument");
    *loop_ms = d->last_ms;
    *steps_run = d->last_steps;
    return TTS_OK;
}

tts_status tts_decoder_resident_limits(tts_decoder* d, int* max_batch, int* max_len) {
    TTS_CHECK(d && max_batch && max_len, TTS_ERR_INVALID, "null argument");
    *max_batch = d->resident ? (d->rbatch ? std::max(1, std::min(d->Bcap, rb_max_batch())) : 1) : 0;
    *max_len = d->resident ? RES_LMAX : 0;
    return TTS_OK;
}

tts_status tts_decoder_last_path(tts_decoder* d, int* resident) {
    TTS_CHECK(d && resident, TTS_ERR_INVALID, "null argument");
    *resident = d->last_resident;
    return TTS_OK;
}

tts_status tts_decoder_resident_phases(tts_decoder* d, float* us, int n) {
    TTS_CHECK(d && us && n >= 2 * RES_PHASES, TTS_ERR_INVALID, "bad arguments");
    long long h[2 * RES_PHASES];
    if (tts_status st = res_rerun(d, true, h)) return st;
    int dev = 0, rate_khz = 1;
    TTS_HIP(hipGetDevice(&dev));
    TTS_HIP(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev));
    for (int i = 0; i < 2 * RES_PHASES; ++i) us[i] = (float)(1e3 * (double)h[i] / rate_khz / d->last_steps);
    return TTS_OK;
}

tts_status tts_decoder_resident_trace(tts_decoder* d, long long* ticks, int64_t n) {
    TTS_CHECK(d && ticks && n >= (int64_t)(RES_PROF_LL - 2 * RES_PHASES), TTS_ERR_INVALID, "bad arguments");
    long long h[2 * RES_PHASES];
    if (tts_status st = res_rerun(d, false, h)) return st;  // no phase marks: only the event stamps
    std::copy(d->res_trace.begin(), d->res_trace.end(), ticks);
    return TTS_OK;
}

tts_status tts_decoder_profile(tts_decoder* d, int reps, float* kernel_ms, int n_kernels) {
    TTS_CHECK(d && kernel_ms && n_kernels >= TTS_DECODER_STEP_KERNELS, TTS_ERR_INVALID, "bad profile arguments");
    TTS_CHECK(d->last_B > 0, TTS_ERR_INVALID, "tts_decoder_profile needs a previous tts_decoder_run");
    // every sentence stays active for the first `last_first` steps: time only those
    reps = std::max(1, std::min(reps, d->last_first - 1));
    const int K = TTS_DECODER_STEP_KERNELS;
    hipEvent_t ev[K + 1];
    for (int i = 0; i <= K; ++i) TTS_HIP(hipEventCreate(&ev[i]));
    TTS_HIP(hipDeviceSynchronize());  // measurement only: nothing else (a pipeline GL) on the device
    hipStream_t s = d->stream;
    InitArgs init = d->last_init;
    if (d->last_enc_direct) {
        // the last run read its encoder output and length in place: stage copies for the step
        // graphs.  The length is the run's own (host record: the device word it read may hold a later
        // sentence's by now, possibly longer than this shape); the encoder rows are read from the
        // caller's buffer as it is now (the caller keeps it alive; the step timings do not depend on
        // its contents)
        const int len = d->last_len_direct;
        TTS_HIP(hipMemcpyAsync(d->enc, d->last_enc_direct, (size_t)d->last_Lmax * ENC * sizeof(float),
                               hipMemcpyDeviceToDevice, s));
        TTS_HIP(hipMemcpyAsync(d->lens, &len, sizeof(int), hipMemcpyHostToDevice, s));
        TTS_HIP(hipStreamSynchronize(s));  // `len` is a stack copy
        init.lens = d->lens;
    }
    TTS_HIP(launch_decoder_init(init, s));
    tts_status st = enqueue_prenet_go(d, d->last_B, s);
    std::vector<double> acc(K, 0.0);
    for (int r = 0; r < reps && st == TTS_OK; ++r) {
        st = enqueue_step(d, d->last_B, d->last_Lmax, d->last_max_steps, r & 1, s, ev);
        if (st) break;
        TTS_HIP(hipEventSynchronize(ev[K]));
        for (int i = 0; i < K; ++i) {
            float ms = 0.f;
            TTS_HIP(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
            acc[i] += ms;
        }
    }
    for (int i = 0; i <= K; ++i) (void)hipEventDestroy(ev[i]);
    if (st) return st;
    for (int i = 0; i < K; ++i) kernel_ms[i] = (float)(acc[i] / reps);
    return TTS_OK;
}

}  // extern "C"

namespace tts {
void decoder_set_pipeline(tts_decoder* d, bool on) {
    d->pipeline = on;
    d->keep_hist = on;
    if (!on) {
        d->post_hook = nullptr;
        decoder_set_pipeline_io(d, nullptr, nullptr, nullptr, nullptr, 0);
    }
}
void decoder_set_pipeline_io(tts_decoder* d, const int* lens_dev, const int* rb_src, int* rb_dst, int* clamp_dst,
                             int clamp_max) {
    d->io_lens = lens_dev;
    d->io_rb_src = rb_src;
    d->io_rb_dst = rb_dst;
    d->io_clamp = clamp_dst;
    d->io_clamp_max = clamp_max;
}
void decoder_set_post_hook(tts_decoder* d, void (*fn)(void*, hipStream_t), void* ctx) {
    d->post_hook = fn;
    d->post_ctx = ctx;
    d->hook_ran = false;
}
bool decoder_hook_ran(tts_decoder* d) { return d->hook_ran && d->last_resident == 1; }
void decoder_histories(tts_decoder* d, const float** mel, int64_t* sentence_floats, const int** n_steps) {
    *mel = d->mel_hist;
    *sentence_floats = (int64_t)d->hist_cap * d->nmel;
    *n_steps = d->n_steps;
}
}  // namespace tts

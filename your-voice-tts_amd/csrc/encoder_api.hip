// Tacotron2 encoder (embedding + Encoder.inference, models/tacotron2.py:63-66,
// layers/tacotron2.py:48-83) as HIP launches replayed from a hipGraph per (B, Lmax):
//   conv 1 with the embedding gather fused into its input staging -> conv 2 -> conv 3
//   (Conv1d k=5 + BatchNorm folded + ReLU, dropout off in eval) -> LSTM input projection for both
//   directions as one KW=1 conv (biases b_ih + b_hh folded) -> Lmax recurrence launches, each a
//   skinny MFMA GEMM over both directions' W_hh with the LSTM cell fused in its epilogue.
// Every sentence is processed at its own length: the convolutions read zeros past L_b and the
// reverse direction starts at L_b - 1, which is what the reference computes running alone.
#include <algorithm>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include <cstdlib>

#include "conv1d.h"
#include "encoder_resident.h"
#include "resident.h"
#include "sgemm.h"

using namespace tts;

namespace {
constexpr int EDIM = 512;  // encoder width
constexpr int EH = 256;    // LSTM hidden per direction
constexpr int EG = 4 * EH; // gate rows per direction
}  // namespace

struct tts_encoder {
    int num_chars = 0, Bcap = 0, Lcap = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev_in = nullptr, ev_out = nullptr;
    std::vector<void*> allocs;
    float* emb = nullptr;
    float* spk = nullptr;  // speaker_embedding.weight [nspk][512] (models/tacotron2.py:32-34), or null
    int nspk = 0;
    float *Wc[3] = {}, *sc[3] = {}, *sh[3] = {};
    float *Wp = nullptr, *bp = nullptr;  // projection [512][1][2048], bias [2048]
    float *Wcf[3] = {}, *Wpf = nullptr;  // fragment-order copies (conv_pack_frag): small-batch conv kernel
    float* Wcf16[3] = {};                // ... in its 16-channel order (conv_pack_frag_tap16), or null
    float* Whh = nullptr;                // packed [2 directions][64 tiles][16 chunks][64][4]
    int *ids = nullptr, *T = nullptr;
    float *act0 = nullptr, *act1 = nullptr, *xi = nullptr, *h = nullptr, *c = nullptr, *out = nullptr;
    float* part = nullptr;  // split-K workspace of the convolutions (CONV_SPLITK_FLOATS)
    std::map<std::pair<int, int>, hipGraphExec_t> graphs;
    // resident batch-1 BiLSTM (encoder_resident.h): one launch for the whole recurrence
    bool resident = false;
    float4* rw = nullptr;
    unsigned long long* rgran = nullptr;
    long long rtmo = 0;
    unsigned rsalt = 0;
    bool rgran_clear = false;  // the resident granules were cleared once (then only on a salt wrap)
    unsigned rsalt_pending = 0;  // salt of the launch whose status a pipeline collects later
    bool pending_batch = false;  // ... and whether it was the batched form
    int* host_status = nullptr;  // pinned
    bool pipeline = false;        // tts_synth_run: caller's stream, placement status left pending
    bool status_pending = false;
    bool defer_status = false;  // pipeline, batch-1 resident: the caller reads the status word back
    bool lens_staged = false;   // pipeline: the caller wrote T on the stream already (stage_ids)
    bool skip_resident_once = false;  // a pipelined resident run timed out: its rerun goes per-step
    int res_timeouts = 0;             // resident runs that timed out a hand-off and re-ran per-step
    std::map<int, hipGraphExec_t> rgraphs;  // by Lmax (B = 1)
    // batched resident BiLSTM (encoder_resident.h, 2 <= B <= 64, no caller state)
    float* whh_raw = nullptr;                // [2][1024][256] W_hh, reference layout
    unsigned long long* bgran = nullptr;     // encoder_resident_batch_granules()
    unsigned bsalt = 0;
    bool bgran_clear = false;
    std::map<std::pair<int, int>, hipGraphExec_t> bgraphs;  // convs + projection, by (B, Lmax)
    int last_resident = 0;                  // the last run's BiLSTM path (tts_encoder_last_path)
};

namespace {

template <typename T>
tts_status emalloc(tts_encoder* e, T** p, size_t n) {
    void* q = nullptr;
    TTS_HIP(hipMalloc(&q, n * sizeof(T) + 16));
    e->allocs.push_back(q);
    *p = static_cast<T*>(q);
    return TTS_OK;
}

tts_status enqueue_encoder(tts_encoder* e, int B, int Lmax, int frames, hipStream_t s, bool resident = false) {
    // outputs past L_b are zero (the batch-1 resident form runs one sentence of length Lmax: it
    // writes every row); the initial LSTM state is set outside the graph (tts_encoder_run_state)
    if (!(resident && B == 1)) TTS_HIP(hipMemsetAsync(e->out, 0, sizeof(float) * (size_t)B * Lmax * EDIM, s));
    float* bufs[2] = {e->act0, e->act1};
    for (int l = 0; l < 3; ++l) {
        ConvArgs a{};
        a.in = l == 0 ? nullptr : bufs[(l - 1) & 1];
        a.ids = l == 0 ? e->ids : nullptr;
        a.table = e->emb;
        a.out = bufs[l & 1];
        a.W = e->Wc[l];
        a.Wf = e->Wcf[l];
        a.Wf16 = e->Wcf16[l];
        a.wf_tap = conv_frag_tap_ok(EDIM) ? 1 : 0;
        a.scale = e->sc[l];
        a.shift = e->sh[l];
        a.T = e->T;
        a.Tmax = Lmax;
        a.Cin = EDIM;
        a.Cout = EDIM;
        a.co_pad = EDIM;
        a.act = CONV_RELU;
        a.part = e->part;
        a.tickets = reinterpret_cast<int*>(e->part + CONV_SPLITK_FLOATS);
        TTS_HIP(conv_launch(a, 5, B, frames, s));
    }
    {
        ConvArgs a{};
        a.in = bufs[0];  // conv 3 output
        a.out = e->xi;
        a.W = e->Wp;
        a.Wf = e->Wpf;
        a.wf_tap = conv_frag_tap_ok(EDIM) ? 1 : 0;
        a.shift = e->bp;
        a.T = e->T;
        a.Tmax = Lmax;
        a.Cin = EDIM;
        a.Cout = 2 * EG;
        a.co_pad = 2 * EG;
        a.act = CONV_NONE;
        a.part = e->part;
        a.tickets = reinterpret_cast<int*>(e->part + CONV_SPLITK_FLOATS);
        TTS_HIP(conv_launch(a, 1, B, frames, s));
    }
    const int64_t hs = (int64_t)e->Bcap * EH;  // per-direction stride; h slots [2][2][Bcap][H]
    if (resident) return TTS_OK;  // the recurrence: enqueue_encoder_resident, launched outside the graph
    for (int st = 0; st < Lmax; ++st) {
        float* h_prev = e->h + (int64_t)((st + 1) & 1) * 2 * hs;
        float* h_next = e->h + (int64_t)(st & 1) * 2 * hs;
        SGemmArgs a{};
        a.B = B;
        a.out_par = -1;
        a.seg[0] = Seg{h_prev, EH, EH};
        a.seg[1] = Seg{h_prev + hs, EH, EH};
        a.nseg = 1;
        a.W = e->Whh;
        a.K = EH;
        a.N = 2 * EG;
        EncLstm& E = a.enc;
        E.tiles_per_dir = EG / 16;
        E.H = EH;
        E.s = st;
        E.lens = e->T;
        E.xi = e->xi;
        E.Tmax = Lmax;
        E.c = e->c;
        E.cstride = hs;
        E.h_next = h_next;
        E.enc_out = e->out;
        TTS_HIP(sgemm_launch(a, ROLE_ENC_LSTM, s));
    }
    return TTS_OK;
}

// B = 1: the whole recurrence in one direct launch (per-launch salt); h_0 / c_0 come from slot 1 / c,
// h_n goes to slot (L-1) & 1 (where tts_encoder_run_state reads it) and c_n to c
tts_status enqueue_encoder_resident(tts_encoder* e, int Lmax, bool zero_state, hipStream_t s, bool* launched) {
    const int64_t hs = (int64_t)e->Bcap * EH;
    bool wrapped = false;
    e->rsalt = res_next_salt(e->rsalt, &wrapped);
    // salted tags and status (resident.h): the granules are cleared once per salt period
    if (wrapped || !e->rgran_clear)
        TTS_HIP(hipMemsetAsync(e->rgran, 0, sizeof(unsigned long long) * encoder_resident_granules(), s));
    e->rgran_clear = true;
    EncResArgs a{};
    a.w = e->rw;
    static const int enc_first_sleep = [] {
        const char* v = getenv("TTS_ENC_FIRST_SLEEP");
        return v ? atoi(v) : 2;  // round 6: ~-9 us per configs[1] sentence (tools/cases_sleep.txt)
    }();
    a.first_sleep = enc_first_sleep;
    a.xi = e->xi;
    a.L = Lmax;
    a.hdir = hs;
    a.h0 = zero_state ? nullptr : e->h + 2 * hs;  // null: the kernel starts from zeros
    a.c0 = zero_state ? nullptr : e->c;
    a.h_fin = e->h + (int64_t)((Lmax - 1) & 1) * 2 * hs;
    a.c_fin = e->c;
    a.out = e->out;
    a.gran = e->rgran;
    a.status = reinterpret_cast<int*>(e->rgran + encoder_resident_granules() - 2);
    a.tmo = e->rtmo;
    a.salt = e->rsalt;
    TTS_HIP(launch_encoder_resident(a, s, launched));
    return TTS_OK;
}

}  // namespace

extern "C" {

void tts_encoder_destroy(tts_encoder* e) {
    if (!e) return;
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    for (auto& kv : e->graphs) (void)hipGraphExecDestroy(kv.second);
    for (auto& kv : e->rgraphs) (void)hipGraphExecDestroy(kv.second);
    for (auto& kv : e->bgraphs) (void)hipGraphExecDestroy(kv.second);
    if (e->host_status) (void)hipHostFree(e->host_status);
    for (void* p : e->allocs) (void)hipFree(p);
    for (hipEvent_t ev : {e->ev_in, e->ev_out})
        if (ev) (void)hipEventDestroy(ev);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

tts_status tts_encoder_create(const tts_tensor* tensors, int n_tensors, int max_batch, int max_len, void* stream,
                              tts_encoder** out) {
    TTS_CHECK(tensors && out, TTS_ERR_INVALID, "null argument");
    TTS_CHECK(max_batch >= 1 && max_batch <= 64, TTS_ERR_UNSUPPORTED, "max_batch must be in [1, 64]");
    TTS_CHECK(max_len >= 1 && max_len <= 4096, TTS_ERR_UNSUPPORTED, "max_len must be in [1, 4096]");
    std::unordered_map<std::string, std::pair<const float*, int64_t>> wm;
    for (int i = 0; i < n_tensors; ++i) wm[tensors[i].key] = {tensors[i].data, tensors[i].numel};
    auto get = [&](const std::string& k, int64_t numel) -> const float* {
        auto it = wm.find(k);
        if (it == wm.end()) { set_error("missing weight " + k); return nullptr; }
        if (numel >= 0 && it->second.second != numel) { set_error("weight " + k + " has wrong size"); return nullptr; }
        return it->second.first;
    };
    auto* e = new tts_encoder();
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto fail = [&](tts_status code) { tts_encoder_destroy(e); return code; };
    tts_status st = TTS_OK;
#define CK(x)                    \
    do {                         \
        st = (x);                \
        if (st) return fail(st); \
    } while (0)
#define HK(x)                                                                    \
    do {                                                                         \
        hipError_t _e = (x);                                                     \
        if (_e != hipSuccess) return fail(hip_fail(_e, #x, __FILE__, __LINE__)); \
    } while (0)
    HK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    HK(hipEventCreateWithFlags(&e->ev_in, hipEventDisableTiming));
    HK(hipEventCreateWithFlags(&e->ev_out, hipEventDisableTiming));
    auto it = wm.find("embedding.weight");
    if (it == wm.end() || it->second.second % EDIM) { set_error("missing/bad embedding.weight"); return fail(TTS_ERR_INVALID); }
    e->num_chars = (int)(it->second.second / EDIM);
    CK(emalloc(e, &e->emb, (size_t)e->num_chars * EDIM));
    HK(hipMemcpyAsync(e->emb, it->second.first, sizeof(float) * e->num_chars * EDIM, hipMemcpyDeviceToDevice, s));
    if (auto sp = wm.find("speaker_embedding.weight"); sp != wm.end()) {
        if (sp->second.second % EDIM || sp->second.second == 0) {
            set_error("bad speaker_embedding.weight");
            return fail(TTS_ERR_INVALID);
        }
        e->nspk = (int)(sp->second.second / EDIM);
        CK(emalloc(e, &e->spk, (size_t)e->nspk * EDIM));
        HK(hipMemcpyAsync(e->spk, sp->second.first, sizeof(float) * e->nspk * EDIM, hipMemcpyDeviceToDevice, s));
    }
    for (int l = 0; l < 3; ++l) {
        const std::string pre = "encoder.convolutions." + std::to_string(l) + ".net.";
        const float* w = get(pre + "0.weight", (int64_t)EDIM * EDIM * 5);
        const float* bias = get(pre + "0.bias", EDIM);
        const float* g = get(pre + "1.weight", EDIM);
        const float* be = get(pre + "1.bias", EDIM);
        const float* mu = get(pre + "1.running_mean", EDIM);
        const float* var = get(pre + "1.running_var", EDIM);
        if (!w || !bias || !g || !be || !mu || !var) return fail(TTS_ERR_INVALID);
        CK(emalloc(e, &e->Wc[l], (size_t)EDIM * 5 * EDIM));
        CK(emalloc(e, &e->sc[l], EDIM));
        CK(emalloc(e, &e->sh[l], EDIM));
        HK(conv_pack(w, EDIM, EDIM, 5, e->Wc[l], s));
        CK(emalloc(e, &e->Wcf[l], (size_t)EDIM * 5 * EDIM));
        HK(conv_frag_tap_ok(EDIM) ? conv_pack_frag_tap(e->Wc[l], EDIM, 5, EDIM, e->Wcf[l], s)
                                  : conv_pack_frag(e->Wc[l], EDIM * 5, EDIM, e->Wcf[l], s));
        if (conv_frag_tap_ok(EDIM)) {
            CK(emalloc(e, &e->Wcf16[l], (size_t)EDIM * 5 * EDIM));
            HK(conv_pack_frag_tap16(e->Wc[l], EDIM, 5, EDIM, e->Wcf16[l], s));
        }
        HK(fold_bn(bias, g, be, mu, var, EDIM, 1e-5f, e->sc[l], e->sh[l], s));
    }
    CK(emalloc(e, &e->Wp, (size_t)EDIM * 2 * EG));
    CK(emalloc(e, &e->bp, 2 * EG));
    CK(emalloc(e, &e->Whh, sgemm_packed_floats(EG, EH) * 2));
    const char* sfx[2] = {"", "_reverse"};
    for (int d = 0; d < 2; ++d) {
        const std::string pre = "encoder.lstm.";
        const float* wih = get(pre + "weight_ih_l0" + sfx[d], (int64_t)EG * EDIM);
        const float* whh = get(pre + "weight_hh_l0" + sfx[d], (int64_t)EG * EH);
        const float* bih = get(pre + "bias_ih_l0" + sfx[d], EG);
        const float* bhh = get(pre + "bias_hh_l0" + sfx[d], EG);
        if (!wih || !whh || !bih || !bhh) return fail(TTS_ERR_INVALID);
        HK(linear_pack_as_conv(wih, EG, EDIM, d * EG, 2 * EG, e->Wp, s));
        // bias: b_ih + b_hh in reference gate order (i, f, g, o) x unit
        HK(sgemm_pack_bias(bih, bhh, EG, ROWMAP_IDENTITY, 0, e->bp + d * EG, s));
        HK(sgemm_pack(whh, EH, nullptr, 0, EG, ROWMAP_LSTM, EH, e->Whh + d * sgemm_packed_floats(EG, EH), s));
    }
    CK(emalloc(e, &e->Wpf, (size_t)EDIM * 2 * EG));
    HK(conv_frag_tap_ok(EDIM) ? conv_pack_frag_tap(e->Wp, EDIM, 1, 2 * EG, e->Wpf, s)
                              : conv_pack_frag(e->Wp, EDIM, 2 * EG, e->Wpf, s));
    e->Bcap = max_batch;
    e->Lcap = max_len;
    const size_t BL = (size_t)max_batch * max_len;
    CK(emalloc(e, &e->ids, BL));
    CK(emalloc(e, &e->T, max_batch));
    CK(emalloc(e, &e->act0, BL * EDIM));
    CK(emalloc(e, &e->act1, BL * EDIM));
    CK(emalloc(e, &e->xi, BL * 2 * EG));
    CK(emalloc(e, &e->h, (size_t)4 * max_batch * EH));
    CK(emalloc(e, &e->c, (size_t)2 * max_batch * EH));
    CK(emalloc(e, &e->out, BL * EDIM));
    CK(emalloc(e, &e->part, CONV_SPLITK_FLOATS + CONV_TICKETS));  // partials, then ticket words (zero at rest)
    HK(hipMemsetAsync(e->part + CONV_SPLITK_FLOATS, 0, CONV_TICKETS * sizeof(int), s));
    {
        const char* env = getenv("TTS_RESIDENT");
        int dev = 0, ncu = 0, rate_khz = 0;
        if (!(env && env[0] == '0') && hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu >= 128 &&
            hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && rate_khz > 0) {
            float* w4 = nullptr;
            CK(emalloc(e, &w4, encoder_resident_weight_float4() * 4));
            e->rw = reinterpret_cast<float4*>(w4);
            CK(emalloc(e, &e->rgran, encoder_resident_granules()));
            HK(encoder_resident_pack(get("encoder.lstm.weight_hh_l0", (int64_t)EG * EH),
                                     get("encoder.lstm.weight_hh_l0_reverse", (int64_t)EG * EH), e->rw, s));
            HK(hipHostMalloc(reinterpret_cast<void**>(&e->host_status), sizeof(int)));
            if (max_batch >= 2) {
                CK(emalloc(e, &e->whh_raw, (size_t)2 * EG * EH));
                HK(hipMemcpyAsync(e->whh_raw, get("encoder.lstm.weight_hh_l0", (int64_t)EG * EH), sizeof(float) * EG * EH,
                                  hipMemcpyDeviceToDevice, s));
                HK(hipMemcpyAsync(e->whh_raw + (size_t)EG * EH, get("encoder.lstm.weight_hh_l0_reverse", (int64_t)EG * EH),
                                  sizeof(float) * EG * EH, hipMemcpyDeviceToDevice, s));
                CK(emalloc(e, &e->bgran, encoder_resident_batch_granules()));
            }
            e->rtmo = (long long)rate_khz * 50;  // 50 ms per hand-off wait
            e->resident = true;
        }
    }
    HK(hipStreamSynchronize(s));
#undef CK
#undef HK
    *out = e;
    return TTS_OK;
}

tts_status tts_encoder_run_state(tts_encoder* e, const int32_t* ids, const int32_t* lens, int B, int Lmax,
                                 const float* state_in, float* state_out, float* out, void* stream) {
    TTS_CHECK(e && ids && lens && out, TTS_ERR_INVALID, "null argument");
    TTS_CHECK(B >= 1 && B <= e->Bcap && Lmax >= 1 && Lmax <= e->Lcap, TTS_ERR_INVALID,
              "batch / length exceeds encoder capacity");
    for (int b = 0; b < B; ++b)
        TTS_CHECK(lens[b] >= 1 && lens[b] <= Lmax, TTS_ERR_INVALID, "length out of range [1, Lmax]");
    hipStream_t cs = static_cast<hipStream_t>(stream);
    hipStream_t s = e->pipeline ? cs : e->stream;
    if (s != cs) {
        TTS_HIP(hipEventRecord(e->ev_in, cs));
        TTS_HIP(hipStreamWaitEvent(s, e->ev_in, 0));
    }
    // (tts_synth_run uploads the ids straight into this handle's buffer: encoder_ids_buffer)
    if (ids != e->ids) TTS_HIP(hipMemcpyAsync(e->ids, ids, sizeof(int) * (size_t)B * Lmax, hipMemcpyDeviceToDevice, s));
    if (!(e->pipeline && e->lens_staged)) TTS_HIP(hipMemcpyAsync(e->T, lens, sizeof(int) * B, hipMemcpyHostToDevice, s));
    // initial state (h_0, c_0) of both directions: step 0 reads the parity-1 h slots
    const size_t hs = (size_t)e->Bcap * EH;  // per-direction stride
    const size_t row = (size_t)B * EH * sizeof(float);
    auto init_state = [&]() -> tts_status {
        if (state_in) {  // [h_fwd, h_bwd, c_fwd, c_bwd] x [B][256]
            for (int d = 0; d < 2; ++d) {
                TTS_HIP(hipMemcpyAsync(e->h + 2 * hs + d * hs, state_in + (size_t)d * B * EH, row,
                                       hipMemcpyDeviceToDevice, s));
                TTS_HIP(hipMemcpyAsync(e->c + d * hs, state_in + (size_t)(2 + d) * B * EH, row,
                                       hipMemcpyDeviceToDevice, s));
            }
        } else {
            TTS_HIP(hipMemsetAsync(e->h, 0, sizeof(float) * 4 * hs, s));
            TTS_HIP(hipMemsetAsync(e->c, 0, sizeof(float) * 2 * hs, s));
        }
        return TTS_OK;
    };
    const bool skip_resident = e->skip_resident_once;
    e->skip_resident_once = false;
    const bool try_resident = e->resident && !skip_resident && B == 1 && lens[0] == Lmax;
    // the resident kernel starts from zeros itself when there is no caller state
    if (!(try_resident && !state_in)) {
        if (tts_status st = init_state()) return st;
    }
    // the batch-1 convs are enqueued directly: a graph launch followed by the resident launch left
    // the GPU idle ~8.7 us between them (configs[1] timeline, round 5); TTS_ENC_GRAPH=1 restores it
    static const bool conv_graph = [] {
        const char* v = getenv("TTS_ENC_GRAPH");
        return v && v[0] == '1';
    }();
    if (try_resident) {
        if (!conv_graph) {
            if (tts_status st = enqueue_encoder(e, 1, Lmax, Lmax, s, true)) return st;
        } else {
            auto rit = e->rgraphs.find(Lmax);
            if (rit == e->rgraphs.end()) {
                hipGraph_t g = nullptr;
                TTS_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
                tts_status st = enqueue_encoder(e, 1, Lmax, Lmax, s, true);
                hipError_t ee = hipStreamEndCapture(s, &g);
                if (st) return st;
                TTS_HIP(ee);
                hipGraphExec_t exec = nullptr;
                TTS_HIP(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0));
                TTS_HIP(hipGraphDestroy(g));
                rit = e->rgraphs.emplace(Lmax, exec).first;
            }
            TTS_HIP(hipGraphLaunch(rit->second, s));
        }
        bool launched = false;
        {
            tts_status st = enqueue_encoder_resident(e, Lmax, !state_in, s, &launched);
            if (st) return st;
        }
        if (!launched) {
            // the grid cannot be co-resident on this device (launch_persistent): nothing ran, the
            // per-step launches below take over for the life of the handle
            e->resident = false;
            if (!state_in) {
                if (tts_status st = init_state()) return st;
            }
        } else {
            e->last_resident = 1;
            e->rsalt_pending = e->rsalt;
            e->pending_batch = false;
            if (!(e->pipeline && e->defer_status))
                TTS_HIP(hipMemcpyAsync(e->host_status, e->rgran + encoder_resident_granules() - 2, sizeof(int),
                                       hipMemcpyDeviceToHost, s));
            if (e->pipeline) {  // the pipeline reads the status at its next synchronisation point
                e->status_pending = true;
                goto done;
            }
            TTS_HIP(hipStreamSynchronize(s));
            e->host_status[0] = res_status_code(e->host_status[0], e->rsalt);
            if (e->host_status[0] == ENC_RES_STATUS_PLACEMENT) {
                e->resident = false;  // rerun below with the per-step launches (same state, untouched)
                if (tts_status st = init_state()) return st;
            } else if (e->host_status[0] != 0) {
                // a hand-off wait timed out (a workgroup could not be placed beside another stream's
                // work): the grid drained; rerun this call with the per-step launches from the
                // initial state (state_in is still the caller's), the handle stays resident
                ++e->res_timeouts;
                if (tts_status st = init_state()) return st;
            } else {
                goto done;
            }
        }
    }
    static const bool batch_off = getenv("TTS_ENC_BATCH_RESIDENT") && getenv("TTS_ENC_BATCH_RESIDENT")[0] == '0';  // A/B knob
    if (e->resident && e->bgran && !skip_resident && B >= 2 && !state_in && !batch_off) {
        // batched resident BiLSTM: the convs + projection graph, then one persistent launch
        auto key = std::make_pair(B, Lmax);
        auto bit = e->bgraphs.find(key);
        if (bit == e->bgraphs.end()) {
            hipGraph_t g = nullptr;
            TTS_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            tts_status st = enqueue_encoder(e, B, Lmax, B * Lmax, s, true);
            hipError_t ee = hipStreamEndCapture(s, &g);
            if (st) return st;
            TTS_HIP(ee);
            hipGraphExec_t exec = nullptr;
            TTS_HIP(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0));
            TTS_HIP(hipGraphDestroy(g));
            bit = e->bgraphs.emplace(key, exec).first;
        }
        TTS_HIP(hipGraphLaunch(bit->second, s));
        bool wrapped = false;
        e->bsalt = res_next_salt(e->bsalt, &wrapped);
        if (wrapped || !e->bgran_clear)
            TTS_HIP(hipMemsetAsync(e->bgran, 0, sizeof(unsigned long long) * encoder_resident_batch_granules(), s));
        e->bgran_clear = true;
        EncResBatchArgs ba{};
        ba.whh = e->whh_raw;
        ba.xi = e->xi;
        ba.lens = e->T;
        ba.B = B;
        ba.Tmax = Lmax;
        ba.out = e->out;
        ba.gran = e->bgran;
        ba.status = reinterpret_cast<int*>(e->bgran + encoder_resident_batch_granules() - 2);
        ba.tmo = e->rtmo;
        ba.salt = e->bsalt;
        bool launched = false;
        TTS_HIP(launch_encoder_resident_batch(ba, s, &launched));
        if (launched) {
            e->last_resident = 2;
            e->rsalt_pending = e->bsalt;
            e->pending_batch = true;
            TTS_HIP(hipMemcpyAsync(e->host_status, ba.status, sizeof(int), hipMemcpyDeviceToHost, s));
            if (e->pipeline) {
                e->status_pending = true;
                goto done;
            }
            TTS_HIP(hipStreamSynchronize(s));
            e->host_status[0] = res_status_code(e->host_status[0], e->bsalt);
            if (e->host_status[0] == 0) goto done;
            // placement failed or a hand-off wait timed out: rerun with the per-step launches
            if (e->host_status[0] == ENC_RES_STATUS_PLACEMENT) e->bgran = nullptr;  // not on this device
            else ++e->res_timeouts;
            if (tts_status st = init_state()) return st;
        }
    }
    {
    auto key = std::make_pair(B, Lmax);
    auto git = e->graphs.find(key);
    if (git == e->graphs.end()) {
        hipGraph_t g = nullptr;
        TTS_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        // tile shape depends on the batch's total frames: key on the worst case (Lmax per sentence)
        tts_status st = enqueue_encoder(e, B, Lmax, B * Lmax, s);
        hipError_t ee = hipStreamEndCapture(s, &g);
        if (st) return st;
        TTS_HIP(ee);
        hipGraphExec_t exec = nullptr;
        TTS_HIP(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0));
        TTS_HIP(hipGraphDestroy(g));
        git = e->graphs.emplace(key, exec).first;
    }
    TTS_HIP(hipGraphLaunch(git->second, s));
    e->last_resident = 0;
    }
done:
    // (tts_synth_run hands this handle's own buffer to the decoder: encoder_out_buffer)
    if (out != e->out) TTS_HIP(hipMemcpyAsync(out, e->out, sizeof(float) * (size_t)B * Lmax * EDIM, hipMemcpyDeviceToDevice, s));
    if (state_out) {
        // h_n of each direction: sentence b wrote its last state at step L_b - 1 (slot (L_b-1) & 1)
        for (int b = 0; b < B; ++b) {
            const float* hsrc = e->h + (size_t)((lens[b] - 1) & 1) * 2 * hs + (size_t)b * EH;
            for (int d = 0; d < 2; ++d) {
                TTS_HIP(hipMemcpyAsync(state_out + ((size_t)d * B + b) * EH, hsrc + d * hs, EH * sizeof(float),
                                       hipMemcpyDeviceToDevice, s));
                TTS_HIP(hipMemcpyAsync(state_out + ((size_t)(2 + d) * B + b) * EH, e->c + d * hs + (size_t)b * EH,
                                       EH * sizeof(float), hipMemcpyDeviceToDevice, s));
            }
        }
    }
    if (s != cs) {
        TTS_HIP(hipEventRecord(e->ev_out, s));
        TTS_HIP(hipStreamWaitEvent(cs, e->ev_out, 0));
    }
    return TTS_OK;
}

}  // extern "C"

namespace tts {
void encoder_set_pipeline(tts_encoder* e, bool on) {
    e->pipeline = on;
    if (!on) e->defer_status = e->lens_staged = false;
}
void encoder_set_lens_staged(tts_encoder* e, bool staged) { e->lens_staged = staged; }
int32_t* encoder_ids_buffer(tts_encoder* e, int B, int Lmax) {
    return (size_t)B * Lmax <= (size_t)e->Bcap * e->Lcap ? e->ids : nullptr;
}
float* encoder_out_buffer(tts_encoder* e) { return e->out; }
const int* encoder_lens_buffer(tts_encoder* e) { return e->T; }
void encoder_status_words(tts_encoder* e, const int** dev, int** host) {
    *dev = e->rgran ? reinterpret_cast<const int*>(e->rgran + encoder_resident_granules() - 2) : nullptr;
    *host = e->host_status;
}
void encoder_set_defer_status(tts_encoder* e, bool defer) { e->defer_status = defer; }

tts_status encoder_pending_status(tts_encoder* e, int* placement_failed) {
    *placement_failed = 0;
    if (!e->status_pending) return TTS_OK;
    e->status_pending = false;  // the caller synchronised the stream the status copy ran on
    e->host_status[0] = res_status_code(e->host_status[0], e->rsalt_pending);
    if (e->host_status[0] == ENC_RES_STATUS_PLACEMENT) {
        if (e->pending_batch) e->bgran = nullptr;  // the batched form cannot be placed on this device
        else e->resident = false;
        *placement_failed = 1;
        return TTS_OK;
    }
    if (e->host_status[0] != 0) {  // a hand-off wait timed out: the caller reruns once per-step
        ++e->res_timeouts;
        e->skip_resident_once = true;
        *placement_failed = 1;
    }
    return TTS_OK;
}
}  // namespace tts

namespace {
// _add_speaker_embedding (models/tacotron2.py:91-100): enc[b][t] += table[speaker[b]] for t < len[b]
struct SpeakerAdd {
    int spk[64];
    int len[64];
};
__global__ void speaker_add_kernel(float* enc, int Lmax, const float* table, const SpeakerAdd a) {
    const int t = blockIdx.x, b = blockIdx.y;
    if (t >= a.len[b]) return;  // rows past the sentence stay zero
    float4* row = reinterpret_cast<float4*>(enc + ((size_t)b * Lmax + t) * EDIM) + threadIdx.x;
    const float4 v = reinterpret_cast<const float4*>(table + (size_t)a.spk[b] * EDIM)[threadIdx.x];
    const float4 x = *row;
    *row = float4{x.x + v.x, x.y + v.y, x.z + v.z, x.w + v.w};
}
}  // namespace

namespace tts {
tts_status encoder_add_speakers(tts_encoder* e, float* enc, const int32_t* lens, const int32_t* speaker_ids, int B,
                                int Lmax, hipStream_t s) {
    TTS_CHECK(e && enc && lens && speaker_ids, TTS_ERR_INVALID, "null argument");
    TTS_CHECK(e->spk, TTS_ERR_INVALID, "speaker embeddings need speaker_embedding.weight at tts_encoder_create");
    TTS_CHECK(B >= 1 && B <= 64 && B <= e->Bcap && Lmax >= 1, TTS_ERR_INVALID, "bad batch for speaker embeddings");
    SpeakerAdd a{};
    for (int b = 0; b < B; ++b) {
        TTS_CHECK(speaker_ids[b] >= 0 && speaker_ids[b] < e->nspk, TTS_ERR_INVALID, "speaker id out of range");
        TTS_CHECK(lens[b] >= 0 && lens[b] <= Lmax, TTS_ERR_INVALID, "length out of range [0, Lmax]");
        a.spk[b] = speaker_ids[b];
        a.len[b] = lens[b];
    }
    hipLaunchKernelGGL(speaker_add_kernel, dim3(Lmax, B), dim3(EDIM / 4), 0, s, enc, Lmax, e->spk, a);
    TTS_HIP(hipGetLastError());
    return TTS_OK;
}
}  // namespace tts

extern "C" {

tts_status tts_encoder_add_speakers(tts_encoder* e, float* enc, const int32_t* lens, const int32_t* speaker_ids, int B,
                                    int Lmax, void* stream) {
    TTS_CHECK(e, TTS_ERR_INVALID, "null argument");
    hipStream_t cs = static_cast<hipStream_t>(stream);
    hipStream_t s = e->pipeline ? cs : e->stream;
    if (s != cs) {
        TTS_HIP(hipEventRecord(e->ev_in, cs));
        TTS_HIP(hipStreamWaitEvent(s, e->ev_in, 0));
    }
    tts_status st = tts::encoder_add_speakers(e, enc, lens, speaker_ids, B, Lmax, s);
    if (st) return st;
    if (s != cs) {
        TTS_HIP(hipEventRecord(e->ev_out, s));
        TTS_HIP(hipStreamWaitEvent(cs, e->ev_out, 0));
    }
    return TTS_OK;
}

tts_status tts_encoder_last_path(tts_encoder* e, int* resident) {
    TTS_CHECK(e && resident, TTS_ERR_INVALID, "null argument");
    *resident = e->last_resident;
    return TTS_OK;
}

tts_status tts_encoder_run(tts_encoder* e, const int32_t* ids, const int32_t* lens, int B, int Lmax, float* out,
                           void* stream) {
    return tts_encoder_run_state(e, ids, lens, B, Lmax, nullptr, nullptr, out, stream);
}

}  // extern "C"

// Tacotron / TacotronGST synthesis path (models/tacotron.py:59-70, models/tacotrongst.py:64-79) for
// gfx950: tts_tacotron_encode (embedding + Prenet + CBHG [+ speaker embedding] [+ GST]),
// tts_tacotron_decode (Decoder.inference, layers/tacotron.py:439-470) and tts_tacotron_postnet
// (PostCBHG + last_linear + sigmoid).
//
// CBHG (layers/tacotron.py:92-206) as MFMA implicit-GEMM convolutions (conv1d.hip):
//   conv bank   ONE conv of K taps: member k's weights centred in the K-tap slab, zeros elsewhere,
//               BatchNorm (eps 1e-3) folded, ReLU;
//   max-pool    fused into the first projection's input staging (max(x[t], x[t+1]), x[T] = 0);
//   projections KW = 3 convs; the last one adds the CBHG input (residual) in its epilogue;
//   [pre_highway] KW = 1 GEMM (PostCBHG only: 80 != 128);
//   highways    one KW = 1 GEMM per layer over interleaved [H | T] rows, gate mix in the epilogue;
//   BiGRU       input projection as one KW = 1 GEMM (b_ih folded), then one persistent workgroup per
//               (sentence, direction) with W_hh in registers (tacotron_kernels.hip).
// GST: six Conv2d + BN + ReLU kernels, GRU input projection (KW = 1 GEMM), the recurrence, and the
// style-token multi-head attention; its output (and the speaker embedding) is added to the
// encoder output in the BiGRU's store.
//
// Decoder step for B sentences, 9 launches (skinny MFMA GEMMs of sgemm.hip + the attention
// kernel), ping-pong buffers bound per step parity, replayed from hipGraphs in chunks:
//   prenet L2 -> attention GRU -> query -> attention (256-wide instance) -> project_to_decoder_in
//   -> decoder GRU 1 (+res) -> decoder GRU 2 (+res) -> proj_to_mel + sigmoid (history, memory)
//   -> [next step's prenet L1 | stopnet + stop rule] (one GEMM over [mel out | decoder out]).
// The stop rule (t > L/4 and (stop > 0.6 or alpha[L-1] > 0.6), or t > max_decoder_steps) runs per
// sentence on the device; the host synchronises once per chunk.
#include <algorithm>
#include <map>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "conv1d.h"
#include "decoder.h"
#include "sgemm.h"
#include "resident.h"
#include "tacotron.h"

using namespace tts;

namespace {

constexpr int NLIN = 1025;  // linear_dim
constexpr int TCHUNK = 16;  // decoder steps per chunk graph

struct Cbhg {
    int K = 0, cin = 0, p0 = 0, p1 = 0;
    float *Wb = nullptr, *scb = nullptr, *shb = nullptr;  // bank slab [cin][K][K*128]
    float *Wp0 = nullptr, *sc0 = nullptr, *sh0 = nullptr;
    float *Wp1 = nullptr, *sc1 = nullptr, *sh1 = nullptr;
    float* Wph = nullptr;  // pre_highway [p1][1][128] or null
    float *Whw[4] = {}, *bhw[4] = {};  // [128][1][256] interleaved H/T, [256]
    float *Wgi = nullptr, *bgi = nullptr;  // GRU input projection [128][1][768], b_ih [768]
    float *Whh = nullptr, *bhh = nullptr;  // [2][384][128], [2][384]
};

struct Buf {
    float* p = nullptr;
    size_t n = 0;
};

struct TGraphs {
    hipGraphExec_t step[2] = {nullptr, nullptr};
    hipGraphExec_t chunk = nullptr;
};

}  // namespace

struct tts_tacotron {
    tts_tacotron_config cfg{};
    int nmel = 400, num_chars = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev_in = nullptr, ev_out = nullptr, ev_t0 = nullptr, ev_t1 = nullptr;
    std::vector<void*> allocs;
    // encoder
    float *emb = nullptr, *Wep0 = nullptr, *bep0 = nullptr, *Wep1 = nullptr, *bep1 = nullptr, *spk = nullptr;
    Cbhg enc, post;
    // GST
    float *gW[6] = {}, *gsc[6] = {}, *gsh[6] = {};
    float *gWi = nullptr, *gbi = nullptr, *gWhh = nullptr, *gbhh = nullptr;
    float *tokens = nullptr, *Wsq = nullptr, *Wsk = nullptr, *Wsv = nullptr;
    // decoder, packed (sgemm.h fragment order)
    float *W_go = nullptr, *b_go = nullptr;    // prenet L1 alone (step 0)
    float *W_p1s = nullptr, *b_p1s = nullptr;  // [prenet L1 | stopnet] over [mel out | decoder out]
    float *W_p2 = nullptr, *b_p2 = nullptr, *W_att = nullptr, *b_att = nullptr, *W_q = nullptr;
    float* W_qT = nullptr;  // query_layer weight transposed [256][128]: the attention launch computes the query
    bool fused_query = true;  // TTS_GST_FUSED_QUERY=0: the separate query GEMM launch (A/B)
    float *W_proj = nullptr, *b_proj = nullptr, *W_g[2] = {}, *b_g[2] = {}, *W_mel = nullptr, *b_mel = nullptr;
    float *v = nullptr, *v_b = nullptr, *ta_w = nullptr, *ta_b = nullptr, *loc_conv = nullptr, *loc_dense = nullptr;
    float *W_in = nullptr, *att_init = nullptr, *dec_init = nullptr, *mem_init = nullptr;
    float *W_ll = nullptr, *b_ll = nullptr;
    // decoder workspace
    int Bcap = 0, Lcap = 0, hist_cap = 0;
    float *denc = nullptr, *Pt = nullptr, *h_att = nullptr, *h1 = nullptr, *h2 = nullptr, *xa = nullptr;
    float *mem = nullptr, *pre1 = nullptr, *q = nullptr, *din = nullptr, *d1 = nullptr, *d2 = nullptr;
    float *alpha = nullptr, *att_w = nullptr, *att_cum = nullptr, *u = nullptr, *tail = nullptr;
    int *lens = nullptr, *win_idx = nullptr, *nidx = nullptr, *flag1 = nullptr, *count = nullptr, *done = nullptr;
    int *n_steps = nullptr, *state = nullptr, *host_flags = nullptr;
    float *mel_hist = nullptr, *stop_hist = nullptr, *align_hist = nullptr;
    std::map<std::tuple<int, int, int>, TGraphs> graphs;
    // sequence workspace (encoder, GST, postnet), grown on demand
    int *ids = nullptr, *T = nullptr, *spk_ids = nullptr, *gT = nullptr;
    Buf bank, p0, y, hwa, hwb, xi, seq_out, pre_a, pre_b, g0, g1, gxi, gh, gst_out, spk_rows;
    // resident decoder (tacotron_resident.hip): raw-layout weight copies, granules, state
    bool resident = false;
    TResArgs rw{};                  // weight pointers (the rest filled per launch)
    unsigned long long* tr_gran = nullptr;  // tres_granules() granules, then the status word
    long long res_ticks = 0;
    unsigned res_salt = 0;
    int res_timeouts = 0, last_resident = 0;
    TResArgs last_ra{};
    // last decode (profiling)
    float last_ms = 0.f;
    int last_steps = 0, last_B = 0, last_Lmax = 0, last_max_steps = 0, last_first = 0;
    TInitArgs last_init{};
};

namespace {

template <typename T>
tts_status talloc(tts_tacotron* t, T** p, size_t n) {
    void* q = nullptr;
    TTS_HIP(hipMalloc(&q, n * sizeof(T) + 16));
    t->allocs.push_back(q);
    *p = static_cast<T*>(q);
    return TTS_OK;
}

// grow-only scratch; frees the old buffer after draining the stream that may still read it
tts_status grow(tts_tacotron* t, Buf& b, size_t n) {
    if (n <= b.n) return TTS_OK;
    if (b.p) {
        TTS_HIP(hipStreamSynchronize(t->stream));
        TTS_HIP(hipFree(b.p));
        b.p = nullptr;
        b.n = 0;
    }
    TTS_HIP(hipMalloc(&b.p, n * sizeof(float) + 16));
    b.n = n;
    return TTS_OK;
}

struct WeightMap {
    std::unordered_map<std::string, std::pair<const float*, int64_t>> m;
    const float* get(const std::string& k, int64_t numel) const {
        auto it = m.find(k);
        if (it == m.end()) {
            set_error("missing weight " + k);
            return nullptr;
        }
        if (numel >= 0 && it->second.second != numel) {
            set_error("weight " + k + " has " + std::to_string(it->second.second) + " elements, expected " +
                      std::to_string(numel));
            return nullptr;
        }
        return it->second.first;
    }
};

tts_status copy_w(tts_tacotron* t, float** dst, const float* src, size_t n, hipStream_t s) {
    tts_status st = talloc(t, dst, n);
    if (st) return st;
    TTS_HIP(hipMemcpyAsync(*dst, src, n * sizeof(float), hipMemcpyDeviceToDevice, s));
    return TTS_OK;
}

#define GET(var, key, n)                         \
    const float* var = wm.get((key), (n));       \
    if (!var) return TTS_ERR_INVALID;

// BatchNorm (eval) of BatchNormConv1d / BatchNorm2d folded into scale / shift
tts_status fold_bn_key(tts_tacotron* t, const WeightMap& wm, const std::string& pre, const float* bias, int C, float eps,
                       float* sc, float* sh, hipStream_t s) {
    GET(g, pre + ".weight", C);
    GET(be, pre + ".bias", C);
    GET(mu, pre + ".running_mean", C);
    GET(var, pre + ".running_var", C);
    TTS_HIP(fold_bn(bias, g, be, mu, var, C, eps, sc, sh, s));
    return TTS_OK;
}

// prenet_type "bn" (common_layers.py:55-70; layers/tacotron.py:283-287): each decoder prenet layer is
// Linear -> BatchNorm1d (eval, eps 1e-5) -> ReLU.  The BatchNorm is folded into the layer's weight
// and bias here, and the folded tensors replace the linear_layer entries, so every consumer (the
// prenet launches, the prenet-1/stop fold, the resident kernel's copies) reads them unchanged.
tts_status fold_prenet_bn(tts_tacotron* t, WeightMap& wm, hipStream_t s) {
    const int outs[2] = {T_PRE1, T_PRE2};
    for (int l = 0; l < 2; ++l) {
        const std::string p = "decoder.prenet.layers." + std::to_string(l) + ".";
        if (!wm.m.count(p + "bn.weight")) {
            if (l == 1 && wm.m.count("decoder.prenet.layers.0.bn.weight")) {
                set_error("missing weight " + p + "bn.weight");
                return TTS_ERR_INVALID;
            }
            continue;
        }
        auto it = wm.m.find(p + "linear_layer.weight");
        if (it == wm.m.end() || it->second.second % outs[l]) {
            set_error("missing or misshapen weight " + p + "linear_layer.weight");
            return TTS_ERR_INVALID;
        }
        const int rows = outs[l], cols = (int)(it->second.second / rows);
        GET(b, p + "linear_layer.bias", rows);
        GET(g, p + "bn.weight", rows);
        GET(be, p + "bn.bias", rows);
        GET(mu, p + "bn.running_mean", rows);
        GET(var, p + "bn.running_var", rows);
        float *wf = nullptr, *bf = nullptr;
        tts_status st = talloc(t, &wf, (size_t)rows * cols);
        if (!st) st = talloc(t, &bf, rows);
        if (st) return st;
        TTS_HIP(fold_linear_bn(it->second.first, b, g, be, mu, var, rows, cols, 1e-5f, wf, bf, s));
        wm.m[p + "linear_layer.weight"] = {wf, (int64_t)rows * cols};
        wm.m[p + "linear_layer.bias"] = {bf, rows};
    }
    return TTS_OK;
}

tts_status make_cbhg(tts_tacotron* t, Cbhg& c, const WeightMap& wm, const std::string& p, int cin, int K, int p0,
                     int p1, hipStream_t s) {
    c.K = K;
    c.cin = cin;
    c.p0 = p0;
    c.p1 = p1;
    const int nb = K * 128;
    tts_status st;
#define CK(x)                \
    do {                     \
        st = (x);            \
        if (st) return st;   \
    } while (0)
    CK(talloc(t, &c.Wb, (size_t)cin * K * nb));
    CK(talloc(t, &c.scb, nb));
    CK(talloc(t, &c.shb, nb));
    TTS_HIP(hipMemsetAsync(c.Wb, 0, sizeof(float) * cin * K * nb, s));
    for (int k = 1; k <= K; ++k) {
        const std::string pre = p + ".conv1d_banks." + std::to_string(k - 1);
        GET(w, pre + ".conv1d.weight", (int64_t)128 * cin * k);
        TTS_HIP(conv_pack_bank(w, 128, cin, k, K, (k - 1) * 128, nb, c.Wb, s));
        CK(fold_bn_key(t, wm, pre + ".bn", nullptr, 128, 1e-3f, c.scb + (k - 1) * 128, c.shb + (k - 1) * 128, s));
    }
    {
        const std::string pre = p + ".conv1d_projections.0";
        GET(w, pre + ".conv1d.weight", (int64_t)p0 * nb * 3);
        CK(talloc(t, &c.Wp0, (size_t)nb * 3 * conv_co_pad(p0)));
        CK(talloc(t, &c.sc0, p0));
        CK(talloc(t, &c.sh0, p0));
        TTS_HIP(conv_pack(w, p0, nb, 3, c.Wp0, s));
        CK(fold_bn_key(t, wm, pre + ".bn", nullptr, p0, 1e-3f, c.sc0, c.sh0, s));
    }
    {
        const std::string pre = p + ".conv1d_projections.1";
        GET(w, pre + ".conv1d.weight", (int64_t)p1 * p0 * 3);
        CK(talloc(t, &c.Wp1, (size_t)p0 * 3 * conv_co_pad(p1)));
        CK(talloc(t, &c.sc1, p1));
        CK(talloc(t, &c.sh1, p1));
        TTS_HIP(conv_pack(w, p1, p0, 3, c.Wp1, s));
        CK(fold_bn_key(t, wm, pre + ".bn", nullptr, p1, 1e-3f, c.sc1, c.sh1, s));
    }
    if (p1 != 128) {
        GET(w, p + ".pre_highway.weight", (int64_t)128 * p1);
        CK(talloc(t, &c.Wph, (size_t)p1 * 128));
        TTS_HIP(linear_pack_as_conv(w, 128, p1, 0, 128, c.Wph, s));
    }
    for (int i = 0; i < 4; ++i) {
        const std::string pre = p + ".highways." + std::to_string(i);
        GET(hw, pre + ".H.weight", 128 * 128);
        GET(hb, pre + ".H.bias", 128);
        GET(tw, pre + ".T.weight", 128 * 128);
        GET(tb, pre + ".T.bias", 128);
        CK(talloc(t, &c.Whw[i], (size_t)128 * 256));
        CK(talloc(t, &c.bhw[i], 256));
        TTS_HIP(linear_pack_strided(hw, 128, 128, 0, 2, 256, c.Whw[i], s));
        TTS_HIP(linear_pack_strided(tw, 128, 128, 1, 2, 256, c.Whw[i], s));
        TTS_HIP(copy_strided(hb, 128, c.bhw[i], 2, s));
        TTS_HIP(copy_strided(tb, 128, c.bhw[i] + 1, 2, s));
    }
    CK(talloc(t, &c.Wgi, (size_t)128 * 768));
    CK(talloc(t, &c.bgi, 768));
    CK(talloc(t, &c.Whh, (size_t)2 * 384 * 128));
    CK(talloc(t, &c.bhh, 768));
    const char* sfx[2] = {"", "_reverse"};
    for (int d = 0; d < 2; ++d) {
        const std::string pre = p + ".gru.";
        GET(wih, pre + "weight_ih_l0" + sfx[d], 384 * 128);
        GET(whh, pre + "weight_hh_l0" + sfx[d], 384 * 128);
        GET(bih, pre + "bias_ih_l0" + sfx[d], 384);
        GET(bhh, pre + "bias_hh_l0" + sfx[d], 384);
        TTS_HIP(linear_pack_as_conv(wih, 384, 128, d * 384, 768, c.Wgi, s));
        TTS_HIP(hipMemcpyAsync(c.bgi + d * 384, bih, 384 * sizeof(float), hipMemcpyDeviceToDevice, s));
        TTS_HIP(hipMemcpyAsync(c.Whh + (size_t)d * 384 * 128, whh, 384 * 128 * sizeof(float), hipMemcpyDeviceToDevice, s));
        TTS_HIP(hipMemcpyAsync(c.bhh + d * 384, bhh, 384 * sizeof(float), hipMemcpyDeviceToDevice, s));
    }
#undef CK
    return TTS_OK;
}

// CBHG.forward over a padded batch: x [B][Tmax][cin] -> out [B][Tmax][256] (rows past T_b untouched)
tts_status run_cbhg(tts_tacotron* t, const Cbhg& c, const float* x, int B, int Tmax, int frames, float* out,
                    const float* add1, const float* add2, hipStream_t s) {
    const size_t BT = (size_t)B * Tmax;
    tts_status st;
    if ((st = grow(t, t->bank, BT * c.K * 128)) || (st = grow(t, t->p0, BT * c.p0)) || (st = grow(t, t->y, BT * c.p1)) ||
        (st = grow(t, t->hwa, BT * 128)) || (st = grow(t, t->hwb, BT * 128)) || (st = grow(t, t->xi, BT * 768)))
        return st;
    ConvArgs a{};
    a.T = t->T;
    a.Tmax = Tmax;
    // conv bank (+ BN + ReLU), all K members in one implicit GEMM
    a.in = x;
    a.out = t->bank.p;
    a.W = c.Wb;
    a.scale = c.scb;
    a.shift = c.shb;
    a.Cin = c.cin;
    a.Cout = c.K * 128;
    a.co_pad = c.K * 128;
    a.act = CONV_RELU;
    TTS_HIP(conv_launch(a, c.K, B, frames, s));
    // max_pool1d fused into the first projection (+ BN + ReLU)
    a = ConvArgs{};
    a.T = t->T;
    a.Tmax = Tmax;
    a.in = t->bank.p;
    a.pool2 = 1;
    a.out = t->p0.p;
    a.W = c.Wp0;
    a.scale = c.sc0;
    a.shift = c.sh0;
    a.Cin = c.K * 128;
    a.Cout = c.p0;
    a.co_pad = conv_co_pad(c.p0);
    a.act = CONV_RELU;
    TTS_HIP(conv_launch(a, 3, B, frames, s));
    // second projection (+ BN), residual x += inputs (layers/tacotron.py:194)
    a.in = t->p0.p;
    a.pool2 = 0;
    a.out = t->y.p;
    a.W = c.Wp1;
    a.scale = c.sc1;
    a.shift = c.sh1;
    a.Cin = c.p0;
    a.Cout = c.p1;
    a.co_pad = conv_co_pad(c.p1);
    a.act = CONV_NONE;
    a.resid = x;
    TTS_HIP(conv_launch(a, 3, B, frames, s));
    const float* cur = t->y.p;
    float* bufs[2] = {t->hwa.p, t->hwb.p};
    int nb = 0;
    if (c.Wph) {  // pre_highway (no bias)
        a = ConvArgs{};
        a.T = t->T;
        a.Tmax = Tmax;
        a.in = cur;
        a.out = bufs[nb];
        a.W = c.Wph;
        a.Cin = c.p1;
        a.Cout = 128;
        a.co_pad = 128;
        a.act = CONV_NONE;
        TTS_HIP(conv_launch(a, 1, B, frames, s));
        cur = bufs[nb];
        nb ^= 1;
    }
    for (int i = 0; i < 4; ++i) {  // Highway: H * T + x * (1 - T)
        a = ConvArgs{};
        a.T = t->T;
        a.Tmax = Tmax;
        a.in = cur;
        a.resid = cur;
        a.out = bufs[nb];
        a.out_ld = 128;
        a.W = c.Whw[i];
        a.shift = c.bhw[i];
        a.Cin = 128;
        a.Cout = 256;
        a.co_pad = 256;
        a.act = CONV_HIGHWAY;
        TTS_HIP(conv_launch(a, 1, B, frames, s));
        cur = bufs[nb];
        nb ^= 1;
    }
    // GRU input projections of both directions (+ b_ih)
    a = ConvArgs{};
    a.T = t->T;
    a.Tmax = Tmax;
    a.in = cur;
    a.out = t->xi.p;
    a.W = c.Wgi;
    a.shift = c.bgi;
    a.Cin = 128;
    a.Cout = 768;
    a.co_pad = 768;
    a.act = CONV_NONE;
    TTS_HIP(conv_launch(a, 1, B, frames, s));
    GruSeqArgs g{};
    g.xi = t->xi.p;
    g.T = t->T;
    g.Tmax = Tmax;
    g.ndir = 2;
    g.Whh = c.Whh;
    g.bhh = c.bhh;
    g.out = out;
    g.out_ld = 256;
    g.add1 = add1;
    g.add2 = add2;
    g.add_ld = 256;
    TTS_HIP(launch_bigru(g, B, s));
    return TTS_OK;
}

// GST(style_mel) -> t->gst_out [B][256]
tts_status run_gst(tts_tacotron* t, const float* style_mel, int Ts, int B, hipStream_t s) {
    static const int filt[7] = {1, 32, 32, 64, 64, 128, 128};
    int H = Ts, W = 80;
    size_t need = 0;
    {
        int h = H, w = W;
        for (int i = 0; i < 6; ++i) {
            h = (h - 1) / 2 + 1;
            w = (w - 1) / 2 + 1;
            need = std::max(need, (size_t)B * filt[i + 1] * h * w);
        }
        TTS_CHECK(128 * w == 256, TTS_ERR_UNSUPPORTED, "GST reference encoder expects 80 mel channels");
    }
    tts_status st;
    if ((st = grow(t, t->g0, need)) || (st = grow(t, t->g1, need))) return st;
    const float* in = style_mel;
    float* bufs[2] = {t->g0.p, t->g1.p};
    for (int i = 0; i < 6; ++i) {
        TTS_HIP(launch_gst_conv2d(in, filt[i], H, W, t->gW[i], t->gsc[i], t->gsh[i], filt[i + 1], bufs[i & 1], i == 5, B,
                                  s));
        in = bufs[i & 1];
        H = (H - 1) / 2 + 1;
        W = (W - 1) / 2 + 1;
    }
    const int H6 = H;
    if ((st = grow(t, t->gxi, (size_t)B * H6 * 384)) || (st = grow(t, t->gh, (size_t)B * 128)) ||
        (st = grow(t, t->gst_out, (size_t)B * 256)))
        return st;
    TTS_HIP(launch_fill_int(t->gT, B, H6, s));
    ConvArgs a{};
    a.in = in;  // [B][H6][256]
    a.out = t->gxi.p;
    a.W = t->gWi;
    a.shift = t->gbi;
    a.T = t->gT;
    a.Tmax = H6;
    a.Cin = 256;
    a.Cout = 384;
    a.co_pad = 384;
    a.act = CONV_NONE;
    TTS_HIP(conv_launch(a, 1, B, B * H6, s));
    GruSeqArgs g{};
    g.xi = t->gxi.p;
    g.T = t->gT;
    g.Tmax = H6;
    g.ndir = 1;
    g.Whh = t->gWhh;
    g.bhh = t->gbhh;
    g.h_last = t->gh.p;
    TTS_HIP(launch_bigru(g, B, s));
    TTS_HIP(launch_style_attention(t->gh.p, t->tokens, t->Wsq, t->Wsk, t->Wsv, t->gst_out.p, B, s));
    return TTS_OK;
}

// Launches of one decoder step of parity p; `ev` (optional, 10 events) brackets every launch.
tts_status enqueue_step(tts_tacotron* t, int B, int Lmax, int max_steps, int p, hipStream_t s,
                        hipEvent_t* ev = nullptr) {
    int mark = 0;
#define MARK() \
    if (ev) TTS_HIP(hipEventRecord(ev[mark++], s));
    const int q = 1 - p;
    const int nmel = t->nmel;
    const int64_t hps = (int64_t)t->Bcap * T_DEC;
    const int64_t xps = (int64_t)t->Bcap * T_XA;
    float* h_att_cur = t->h_att + p * hps;
    float* h_att_prev = t->h_att + q * hps;
    float* h1_cur = t->h1 + p * hps;
    float* h1_prev = t->h1 + q * hps;
    float* h2_cur = t->h2 + p * hps;
    float* h2_prev = t->h2 + q * hps;
    float* xa_cur = t->xa + p * xps;               // [prenet_t | ctx_{t-1}]
    float* ctx_cur = t->xa + q * xps + T_PRE2;     // ctx_t (row stride T_XA)
    int* st_cur = t->state + 2 * p;
    SGemmArgs g{};
    g.B = B;
    g.step = st_cur;
    g.done = t->done;
    g.out_par = -1;
    {  // 1) prenet layer 2 (common_layers.py:77-83) -> xa_cur[0:128]
        SGemmArgs a = g;
        a.seg[0] = Seg{t->pre1, T_PRE1, T_PRE1};
        a.nseg = 1;
        a.W = t->W_p2; a.K = T_PRE1; a.N = T_PRE2; a.bias = t->b_p2; a.act = ACT_RELU;
        a.out = xa_cur; a.ldo = T_XA;
        MARK();
        TTS_HIP(sgemm_launch(a, ROLE_T_PRENET2, s));
    }
    {  // 2) attention GRU: x = [prenet_t | ctx_{t-1}], h = h_att_{t-1} (layers/tacotron.py:370)
        SGemmArgs a = g;
        a.seg[0] = Seg{xa_cur, T_XA, T_XA};
        a.seg[1] = Seg{h_att_prev, T_DEC, T_DEC};
        a.nseg = 2;
        a.W = t->W_att; a.K = T_XA + T_DEC; a.N = 4 * T_DEC; a.bias = t->b_att;
        a.out = h_att_cur; a.ldo = T_DEC;
        a.gru = GruEpi{h_att_prev, T_DEC, nullptr, 0, nullptr, 0};
        MARK();
        TTS_HIP(sgemm_launch(a, ROLE_T_ATT_GRU, s));
    }
    {  // 3) processed query = query_layer(h_att_t) (common_layers.py:179): inside the attention
        // launch (fused_query) or its own GEMM; the profiling mark stays so the per-kernel events
        // keep their order (the fused query's time is in the attention interval)
        MARK();
        if (!t->fused_query) {
            SGemmArgs a = g;
            a.seg[0] = Seg{h_att_cur, T_DEC, T_DEC};
            a.nseg = 1;
            a.W = t->W_q; a.K = T_DEC; a.N = ADIM;
            a.out = t->q; a.ldo = ADIM;
            TTS_HIP(sgemm_launch(a, ROLE_T_QUERY, s));
        }
    }
    {  // 4) attention (energies, norm, forward attention, context -> ctx_t), :371
        const tts_tacotron_config& c = t->cfg;
        AttnArgs a{};
        a.attn_norm = c.attn_norm; a.forward_attn = c.forward_attn; a.trans_agent = c.trans_agent;
        a.forward_attn_mask = c.forward_attn_mask; a.location_attn = c.location_attn; a.windowing = c.windowing;
        a.Lcap = t->Lcap; a.B = B; a.enc_dim = T_DEC; a.ctx_ld = T_XA; a.tail_rule = 1;
        a.v = t->v; a.v_b = t->v_b; a.ta_w = t->ta_w; a.ta_b = t->ta_b;
        a.loc_conv = t->loc_conv; a.loc_dense = t->loc_dense;
        a.q = t->q; a.Pt = t->Pt; a.enc = t->denc; a.lens = t->lens;
        a.wqT = t->fused_query ? t->W_qT : nullptr;
        a.h_att = h_att_cur;  // (no epart: the launch evaluates the energies, attention_kernel<256, 256>)
        a.alpha = t->alpha; a.att_w = t->att_w; a.att_cum = t->att_cum; a.u = t->u; a.win_idx = t->win_idx;
        a.nidx = t->nidx; a.tail = t->tail;
        a.ctx = ctx_cur;
        a.align_hist = t->align_hist; a.align_ldb = (int64_t)t->hist_cap * Lmax; a.Lalign = Lmax;
        a.hist_cap = t->hist_cap;
        a.step = st_cur; a.done = t->done;
        MARK();
        TTS_HIP(launch_attention(a, s));
    }
    {  // 5) project_to_decoder_in([h_att | ctx]) (:373-375)
        SGemmArgs a = g;
        a.seg[0] = Seg{h_att_cur, T_DEC, T_DEC};
        a.seg[1] = Seg{ctx_cur, T_XA, T_DEC};
        a.nseg = 2;
        a.W = t->W_proj; a.K = 2 * T_DEC; a.N = T_DEC; a.bias = t->b_proj;
        a.out = t->din; a.ldo = T_DEC;
        MARK();
        TTS_HIP(sgemm_launch(a, ROLE_T_PROJ, s));
    }
    {  // 6) decoder GRU 1 + residual (:377-381)
        SGemmArgs a = g;
        a.seg[0] = Seg{t->din, T_DEC, T_DEC};
        a.seg[1] = Seg{h1_prev, T_DEC, T_DEC};
        a.nseg = 2;
        a.W = t->W_g[0]; a.K = 2 * T_DEC; a.N = 4 * T_DEC; a.bias = t->b_g[0];
        a.out = h1_cur; a.ldo = T_DEC;
        a.gru = GruEpi{h1_prev, T_DEC, t->din, T_DEC, t->d1, T_DEC};
        MARK();
        TTS_HIP(sgemm_launch(a, ROLE_T_DEC_GRU, s));
    }
    {  // 7) decoder GRU 2 + residual
        SGemmArgs a = g;
        a.seg[0] = Seg{t->d1, T_DEC, T_DEC};
        a.seg[1] = Seg{h2_prev, T_DEC, T_DEC};
        a.nseg = 2;
        a.W = t->W_g[1]; a.K = 2 * T_DEC; a.N = 4 * T_DEC; a.bias = t->b_g[1];
        a.out = h2_cur; a.ldo = T_DEC;
        a.gru = GruEpi{h2_prev, T_DEC, t->d1, T_DEC, t->d2, T_DEC};
        MARK();
        TTS_HIP(sgemm_launch(a, ROLE_T_DEC_GRU, s));
    }
    {  // 8) output = sigmoid(proj_to_mel(decoder_output)) -> history + next memory (:385-386, 396-404)
        SGemmArgs a = g;
        a.seg[0] = Seg{t->d2, T_DEC, T_DEC};
        a.nseg = 1;
        a.W = t->W_mel; a.K = T_DEC; a.N = nmel; a.bias = t->b_mel; a.act = ACT_SIGMOID;
        a.out = t->mem; a.ldo = nmel;
        a.hist = t->mel_hist; a.ldh = (int64_t)t->hist_cap * nmel; a.hist_cap = t->hist_cap;
        MARK();
        TTS_HIP(sgemm_launch(a, ROLE_T_MEL, s));
    }
    {  // 9) next step's prenet L1 over the output, stopnet over [decoder_output | output] + stop rule
        SGemmArgs a = g;
        a.seg[0] = Seg{t->mem, nmel, nmel};
        a.seg[1] = Seg{t->d2, T_DEC, T_DEC};
        a.nseg = 2;
        a.W = t->W_p1s; a.K = nmel + T_DEC; a.N = T_PRE1 + 1; a.bias = t->b_p1s;
        a.hist = t->mel_hist; a.ldh = (int64_t)t->hist_cap * nmel; a.hist_cap = t->hist_cap;  // enables stop history
        MelFused& m = a.mf;
        m.nmel = 0; m.pre1 = t->pre1; m.ldp = T_PRE1;
        m.stop_hist = t->stop_hist; m.stop_ldb = t->hist_cap;
        m.lens = t->lens; m.tail = t->tail; m.flag1 = t->flag1; m.count = t->count;
        m.done = t->done; m.n_steps = t->n_steps;
        m.state_next = t->state + 2 * q;
        m.stop_acc = t->state + 4;
        m.max_steps = max_steps;
        m.rule = 1;
        MARK();
        TTS_HIP(sgemm_launch(a, ROLE_T_PRE1_STOP, s));
    }
    MARK();
#undef MARK
    return TTS_OK;
}

tts_status build_graph(tts_tacotron* t, int B, int Lmax, int max_steps, int first_parity, int steps,
                       hipGraphExec_t* out) {
    hipGraph_t g = nullptr;
    TTS_HIP(hipStreamBeginCapture(t->stream, hipStreamCaptureModeThreadLocal));
    tts_status st = TTS_OK;
    for (int i = 0; i < steps && st == TTS_OK; ++i) st = enqueue_step(t, B, Lmax, max_steps, (first_parity + i) & 1, t->stream);
    hipError_t e = hipStreamEndCapture(t->stream, &g);
    if (st) return st;
    TTS_HIP(e);
    TTS_HIP(hipGraphInstantiate(out, g, nullptr, nullptr, 0));
    TTS_HIP(hipGraphDestroy(g));
    return TTS_OK;
}

// step-0 prenet layer 1 on memory_init (later steps get it from launch 9)
tts_status enqueue_prenet_go(tts_tacotron* t, int B, hipStream_t s) {
    SGemmArgs a{};
    a.B = B;
    a.step = t->state;
    a.out_par = -1;
    a.seg[0] = Seg{t->mem, t->nmel, t->nmel};
    a.nseg = 1;
    a.W = t->W_go; a.K = t->nmel; a.N = T_PRE1; a.bias = t->b_go; a.act = ACT_RELU;
    a.out = t->pre1; a.ldo = T_PRE1;
    TTS_HIP(sgemm_launch(a, ROLE_T_PRENET1, s));
    return TTS_OK;
}

tts_status pack_linear(tts_tacotron* t, const float* W, int N, int K, float** dst, hipStream_t s) {
    tts_status st = talloc(t, dst, sgemm_packed_floats(N, K));
    if (st) return st;
    TTS_HIP(sgemm_pack(W, K, nullptr, 0, N, ROWMAP_IDENTITY, 0, *dst, s));
    return TTS_OK;
}

tts_status pack_bias(tts_tacotron* t, const float* a, const float* b, int N, int rowmap, int H, float** dst,
                     hipStream_t s) {
    tts_status st = talloc(t, dst, (size_t)(N + 15) / 16 * 16);
    if (st) return st;
    TTS_HIP(sgemm_pack_bias(a, b, N, rowmap, H, *dst, s));
    return TTS_OK;
}

tts_status create_weights(tts_tacotron* t, const WeightMap& wm, hipStream_t s) {
    const tts_tacotron_config& c = t->cfg;
    const int nmel = t->nmel;
    tts_status st;
#define CK(x)              \
    do {                   \
        st = (x);          \
        if (st) return st; \
    } while (0)
    // ---- encoder: embedding, prenet, CBHG(K=16, [128, 128])
    {
        auto it = wm.m.find("embedding.weight");
        if (it == wm.m.end() || it->second.second % 256) {
            set_error("missing/bad embedding.weight");
            return TTS_ERR_INVALID;
        }
        t->num_chars = (int)(it->second.second / 256);
        CK(copy_w(t, &t->emb, it->second.first, (size_t)t->num_chars * 256, s));
    }
    if (c.num_speakers > 1) {
        GET(w, "speaker_embedding.weight", (int64_t)c.num_speakers * 256);
        CK(copy_w(t, &t->spk, w, (size_t)c.num_speakers * 256, s));
    }
    {
        GET(w0, "encoder.prenet.layers.0.linear_layer.weight", 256 * 256);
        GET(b0, "encoder.prenet.layers.0.linear_layer.bias", 256);
        GET(w1, "encoder.prenet.layers.1.linear_layer.weight", 128 * 256);
        GET(b1, "encoder.prenet.layers.1.linear_layer.bias", 128);
        CK(talloc(t, &t->Wep0, (size_t)256 * 256));
        CK(talloc(t, &t->Wep1, (size_t)256 * 128));
        TTS_HIP(linear_pack_as_conv(w0, 256, 256, 0, 256, t->Wep0, s));
        TTS_HIP(linear_pack_as_conv(w1, 128, 256, 0, 128, t->Wep1, s));
        CK(copy_w(t, &t->bep0, b0, 256, s));
        CK(copy_w(t, &t->bep1, b1, 128, s));
    }
    CK(make_cbhg(t, t->enc, wm, "encoder.cbhg.cbhg", 128, 16, 128, 128, s));
    // ---- GST
    if (c.gst) {
        static const int filt[7] = {1, 32, 32, 64, 64, 128, 128};
        for (int i = 0; i < 6; ++i) {
            const std::string pre = "gst.encoder.convs." + std::to_string(i);
            const int64_t n = (int64_t)filt[i + 1] * filt[i] * 9;
            GET(w, pre + ".weight", n);
            GET(bias, pre + ".bias", filt[i + 1]);
            CK(copy_w(t, &t->gW[i], w, n, s));
            CK(talloc(t, &t->gsc[i], filt[i + 1]));
            CK(talloc(t, &t->gsh[i], filt[i + 1]));
            CK(fold_bn_key(t, wm, "gst.encoder.bns." + std::to_string(i), bias, filt[i + 1], 1e-5f, t->gsc[i], t->gsh[i],
                           s));
        }
        GET(wih, "gst.encoder.recurrence.weight_ih_l0", 384 * 256);
        GET(whh, "gst.encoder.recurrence.weight_hh_l0", 384 * 128);
        GET(bih, "gst.encoder.recurrence.bias_ih_l0", 384);
        GET(bhh, "gst.encoder.recurrence.bias_hh_l0", 384);
        CK(talloc(t, &t->gWi, (size_t)256 * 384));
        TTS_HIP(linear_pack_as_conv(wih, 384, 256, 0, 384, t->gWi, s));
        CK(copy_w(t, &t->gbi, bih, 384, s));
        CK(copy_w(t, &t->gWhh, whh, 384 * 128, s));
        CK(copy_w(t, &t->gbhh, bhh, 384, s));
        GET(tok, "gst.style_token_layer.style_tokens", 10 * 64);
        GET(wq, "gst.style_token_layer.attention.W_query.weight", 256 * 128);
        GET(wk, "gst.style_token_layer.attention.W_key.weight", 256 * 64);
        GET(wv, "gst.style_token_layer.attention.W_value.weight", 256 * 64);
        CK(copy_w(t, &t->tokens, tok, 640, s));
        CK(copy_w(t, &t->Wsq, wq, 256 * 128, s));
        CK(copy_w(t, &t->Wsk, wk, 256 * 64, s));
        CK(copy_w(t, &t->Wsv, wv, 256 * 64, s));
    }
    // ---- decoder
    {
        GET(pw0, "decoder.prenet.layers.0.linear_layer.weight", (int64_t)T_PRE1 * nmel);
        GET(pb0, "decoder.prenet.layers.0.linear_layer.bias", T_PRE1);
        GET(pw1, "decoder.prenet.layers.1.linear_layer.weight", T_PRE2 * T_PRE1);
        GET(pb1, "decoder.prenet.layers.1.linear_layer.bias", T_PRE2);
        GET(sw, "decoder.stopnet.linear.weight", T_DEC + nmel);
        GET(sb, "decoder.stopnet.linear.bias", 1);
        CK(pack_linear(t, pw0, T_PRE1, nmel, &t->W_go, s));
        CK(pack_bias(t, pb0, nullptr, T_PRE1, ROWMAP_IDENTITY, 0, &t->b_go, s));
        CK(pack_linear(t, pw1, T_PRE2, T_PRE1, &t->W_p2, s));
        CK(pack_bias(t, pb1, nullptr, T_PRE2, ROWMAP_IDENTITY, 0, &t->b_p2, s));
        float *wf = nullptr, *bf = nullptr;
        const int K = nmel + T_DEC;
        TTS_HIP(hipMalloc(&wf, sizeof(float) * (T_PRE1 + 1) * K));
        TTS_HIP(hipMalloc(&bf, sizeof(float) * (T_PRE1 + 1)));
        hipError_t e = fold_pre1_stop(pw0, pb0, sw, sb, nmel, wf, bf, s);
        if (e == hipSuccess) st = pack_linear(t, wf, T_PRE1 + 1, K, &t->W_p1s, s);
        if (e == hipSuccess && !st) st = pack_bias(t, bf, nullptr, T_PRE1 + 1, ROWMAP_IDENTITY, 0, &t->b_p1s, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        (void)hipFree(wf);
        (void)hipFree(bf);
        TTS_HIP(e);
        if (st) return st;
    }
    {
        GET(wih, "decoder.attention_rnn.weight_ih", (int64_t)3 * T_DEC * T_XA);
        GET(whh, "decoder.attention_rnn.weight_hh", (int64_t)3 * T_DEC * T_DEC);
        GET(bih, "decoder.attention_rnn.bias_ih", 3 * T_DEC);
        GET(bhh, "decoder.attention_rnn.bias_hh", 3 * T_DEC);
        CK(talloc(t, &t->W_att, sgemm_packed_floats(4 * T_DEC, T_XA + T_DEC)));
        TTS_HIP(sgemm_pack(wih, T_XA, whh, T_DEC, 4 * T_DEC, ROWMAP_GRU, T_DEC, t->W_att, s));
        CK(pack_bias(t, bih, bhh, 4 * T_DEC, ROWMAP_GRU, T_DEC, &t->b_att, s));
    }
    {
        GET(wq, "decoder.attention_layer.query_layer.linear_layer.weight", ADIM * T_DEC);
        GET(win, "decoder.attention_layer.inputs_layer.linear_layer.weight", ADIM * T_DEC);
        GET(vw, "decoder.attention_layer.v.linear_layer.weight", ADIM);
        GET(vb, "decoder.attention_layer.v.linear_layer.bias", 1);
        CK(pack_linear(t, wq, ADIM, T_DEC, &t->W_q, s));
        CK(talloc(t, &t->W_qT, (size_t)ADIM * T_DEC));
        TTS_HIP(transpose_f32(wq, ADIM, T_DEC, t->W_qT, s));
        {
            const char* fq = getenv("TTS_GST_FUSED_QUERY");
            t->fused_query = !(fq && fq[0] == '0');
        }
        CK(copy_w(t, &t->W_in, win, ADIM * T_DEC, s));
        CK(copy_w(t, &t->v, vw, ADIM, s));
        CK(copy_w(t, &t->v_b, vb, 1, s));
        if (c.trans_agent) {
            GET(taw, "decoder.attention_layer.ta.weight", 2 * T_DEC);
            GET(tab, "decoder.attention_layer.ta.bias", 1);
            CK(copy_w(t, &t->ta_w, taw, 2 * T_DEC, s));
            CK(copy_w(t, &t->ta_b, tab, 1, s));
        }
        if (c.location_attn) {
            GET(lcw, "decoder.attention_layer.location_layer.location_conv.weight", NLOC * 2 * KLOC);
            GET(ldw, "decoder.attention_layer.location_layer.location_dense.linear_layer.weight", ADIM * NLOC);
            CK(copy_w(t, &t->loc_conv, lcw, NLOC * 2 * KLOC, s));
            CK(copy_w(t, &t->loc_dense, ldw, ADIM * NLOC, s));
        }
    }
    {
        GET(pw, "decoder.project_to_decoder_in.weight", T_DEC * 2 * T_DEC);
        GET(pb, "decoder.project_to_decoder_in.bias", T_DEC);
        CK(pack_linear(t, pw, T_DEC, 2 * T_DEC, &t->W_proj, s));
        CK(pack_bias(t, pb, nullptr, T_DEC, ROWMAP_IDENTITY, 0, &t->b_proj, s));
        for (int i = 0; i < 2; ++i) {
            const std::string pre = "decoder.decoder_rnns." + std::to_string(i) + ".";
            GET(wih, pre + "weight_ih", 3 * T_DEC * T_DEC);
            GET(whh, pre + "weight_hh", 3 * T_DEC * T_DEC);
            GET(bih, pre + "bias_ih", 3 * T_DEC);
            GET(bhh, pre + "bias_hh", 3 * T_DEC);
            CK(talloc(t, &t->W_g[i], sgemm_packed_floats(4 * T_DEC, 2 * T_DEC)));
            TTS_HIP(sgemm_pack(wih, T_DEC, whh, T_DEC, 4 * T_DEC, ROWMAP_GRU, T_DEC, t->W_g[i], s));
            CK(pack_bias(t, bih, bhh, 4 * T_DEC, ROWMAP_GRU, T_DEC, &t->b_g[i], s));
        }
        GET(mw, "decoder.proj_to_mel.weight", (int64_t)nmel * T_DEC);
        GET(mb, "decoder.proj_to_mel.bias", nmel);
        CK(pack_linear(t, mw, nmel, T_DEC, &t->W_mel, s));
        CK(pack_bias(t, mb, nullptr, nmel, ROWMAP_IDENTITY, 0, &t->b_mel, s));
        GET(ai, "decoder.attention_rnn_init.weight", T_DEC);
        GET(mi, "decoder.memory_init.weight", nmel);
        GET(di, "decoder.decoder_rnn_inits.weight", 2 * T_DEC);
        CK(copy_w(t, &t->att_init, ai, T_DEC, s));
        CK(copy_w(t, &t->mem_init, mi, nmel, s));
        CK(copy_w(t, &t->dec_init, di, 2 * T_DEC, s));
    }
    // ---- PostCBHG(K=8, [256, 80]) + last_linear
    CK(make_cbhg(t, t->post, wm, "postnet.cbhg", 80, 8, 256, 80, s));
    {
        GET(lw, "last_linear.0.weight", (int64_t)NLIN * 256);
        GET(lb, "last_linear.0.bias", NLIN);
        CK(talloc(t, &t->W_ll, (size_t)256 * conv_co_pad(NLIN)));
        TTS_HIP(hipMemsetAsync(t->W_ll, 0, sizeof(float) * 256 * conv_co_pad(NLIN), s));
        TTS_HIP(linear_pack_as_conv(lw, NLIN, 256, 0, conv_co_pad(NLIN), t->W_ll, s));
        CK(copy_w(t, &t->b_ll, lb, NLIN, s));
    }
#undef CK
    return TTS_OK;
}

tts_status create_workspace(tts_tacotron* t, hipStream_t s) {
    const tts_tacotron_config& c = t->cfg;
    const int Bc = c.max_batch, Lc = (c.max_len + 3) / 4 * 4;
    t->Bcap = Bc;
    t->Lcap = Lc;
    t->hist_cap = c.max_steps + 1;
    tts_status st;
#define CK(x)              \
    do {                   \
        st = (x);          \
        if (st) return st; \
    } while (0)
    CK(talloc(t, &t->denc, (size_t)Bc * Lc * T_DEC));
    CK(talloc(t, &t->Pt, (size_t)Bc * ADIM * Lc));
    CK(talloc(t, &t->h_att, (size_t)2 * Bc * T_DEC));
    CK(talloc(t, &t->h1, (size_t)2 * Bc * T_DEC));
    CK(talloc(t, &t->h2, (size_t)2 * Bc * T_DEC));
    CK(talloc(t, &t->xa, (size_t)2 * Bc * T_XA));
    CK(talloc(t, &t->mem, (size_t)Bc * t->nmel));
    CK(talloc(t, &t->pre1, (size_t)Bc * T_PRE1));
    CK(talloc(t, &t->q, (size_t)Bc * ADIM));
    CK(talloc(t, &t->din, (size_t)Bc * T_DEC));
    CK(talloc(t, &t->d1, (size_t)Bc * T_DEC));
    CK(talloc(t, &t->d2, (size_t)Bc * T_DEC));
    CK(talloc(t, &t->alpha, (size_t)Bc * Lc));
    CK(talloc(t, &t->att_w, (size_t)Bc * Lc));
    CK(talloc(t, &t->att_cum, (size_t)Bc * Lc));
    CK(talloc(t, &t->u, Bc));
    CK(talloc(t, &t->tail, Bc));
    CK(talloc(t, &t->lens, Bc));
    CK(talloc(t, &t->win_idx, Bc));
    CK(talloc(t, &t->nidx, Bc));
    CK(talloc(t, &t->flag1, Bc));
    CK(talloc(t, &t->count, Bc));
    CK(talloc(t, &t->done, Bc));
    CK(talloc(t, &t->n_steps, Bc));
    CK(talloc(t, &t->state, 8));  // {step, n_active} x 2 parities, stop_acc
    CK(talloc(t, &t->mel_hist, (size_t)Bc * t->hist_cap * t->nmel));
    CK(talloc(t, &t->stop_hist, (size_t)Bc * t->hist_cap));
    CK(talloc(t, &t->align_hist, (size_t)Bc * t->hist_cap * Lc));
    CK(talloc(t, &t->ids, (size_t)Bc * std::max(Lc, 1)));
    CK(talloc(t, &t->T, Bc));
    CK(talloc(t, &t->spk_ids, Bc));
    CK(talloc(t, &t->gT, Bc));
#undef CK
    TTS_HIP(attention_prepare(Lc, c.location_attn));
    TTS_HIP(hipMemsetAsync(t->xa, 0, sizeof(float) * 2 * Bc * T_XA, s));
    TTS_HIP(hipMemsetAsync(t->d2, 0, sizeof(float) * Bc * T_DEC, s));
    TTS_HIP(hipMemsetAsync(t->denc, 0, sizeof(float) * Bc * Lc * T_DEC, s));
    TTS_HIP(hipMemsetAsync(t->Pt, 0, sizeof(float) * Bc * ADIM * Lc, s));
    TTS_HIP(hipMemsetAsync(t->state, 0, sizeof(int) * 8, s));
    return TTS_OK;
}

// The resident decoder serves the attention configuration of config_tacotron_gst.json (sigmoid norm,
// forward attention without the eval mask, no transition agent / location / windowing) on a GPU
// with >= 256 compute units; TTS_RESIDENT=0 at create disables it.  Its weights are plain copies of
// the reference tensors (the kernel picks its rows at launch).
tts_status create_resident(tts_tacotron* t, const WeightMap& wm, hipStream_t s) {
    const tts_tacotron_config& c = t->cfg;
    const char* env = getenv("TTS_RESIDENT");
    int dev = 0, ncu = 0, rate_khz = 0;
    if (!(c.attn_norm == 1 && c.forward_attn && !c.trans_agent && !c.forward_attn_mask && !c.location_attn &&
          !c.windowing && t->nmel <= TR_NMEL_MAX && c.max_steps <= 1000) ||
        (env && env[0] == '0') || hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < TR_CUS ||
        hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || rate_khz <= 0 ||
        tres_prepare() != hipSuccess)
        return TTS_OK;
    const int nmel = t->nmel;
    TResArgs& a = t->rw;
    tts_status st;
#define CPY(dst, key, n)                      \
    do {                                      \
        GET(src_, key, n);                    \
        float* d_ = nullptr;                  \
        if ((st = copy_w(t, &d_, src_, (size_t)(n), s))) return st; \
        dst = d_;                             \
    } while (0)
    CPY(a.a_wih, "decoder.attention_rnn.weight_ih", (int64_t)3 * T_DEC * T_XA);
    CPY(a.a_whh, "decoder.attention_rnn.weight_hh", (int64_t)3 * T_DEC * T_DEC);
    CPY(a.a_bih, "decoder.attention_rnn.bias_ih", 3 * T_DEC);
    CPY(a.a_bhh, "decoder.attention_rnn.bias_hh", 3 * T_DEC);
    for (int i = 0; i < 2; ++i) {
        const std::string pre = "decoder.decoder_rnns." + std::to_string(i) + ".";
        CPY(a.g_wih[i], pre + "weight_ih", 3 * T_DEC * T_DEC);
        CPY(a.g_whh[i], pre + "weight_hh", 3 * T_DEC * T_DEC);
        CPY(a.g_bih[i], pre + "bias_ih", 3 * T_DEC);
        CPY(a.g_bhh[i], pre + "bias_hh", 3 * T_DEC);
    }
    CPY(a.w_proj, "decoder.project_to_decoder_in.weight", T_DEC * 2 * T_DEC);
    CPY(a.b_proj, "decoder.project_to_decoder_in.bias", T_DEC);
    CPY(a.w_mel, "decoder.proj_to_mel.weight", (int64_t)nmel * T_DEC);
    CPY(a.b_mel, "decoder.proj_to_mel.bias", nmel);
    CPY(a.w_pre1, "decoder.prenet.layers.0.linear_layer.weight", (int64_t)T_PRE1 * nmel);
    CPY(a.b_pre1, "decoder.prenet.layers.0.linear_layer.bias", T_PRE1);
    CPY(a.w_pre2, "decoder.prenet.layers.1.linear_layer.weight", T_PRE2 * T_PRE1);
    CPY(a.b_pre2, "decoder.prenet.layers.1.linear_layer.bias", T_PRE2);
    CPY(a.w_q, "decoder.attention_layer.query_layer.linear_layer.weight", ADIM * T_DEC);
    CPY(a.w_stop, "decoder.stopnet.linear.weight", T_DEC + nmel);
    CPY(a.b_stop, "decoder.stopnet.linear.bias", 1);
#undef CPY
    a.v = t->v;
    a.v_b = t->v_b;
    if ((st = talloc(t, &t->tr_gran, tres_granules() + 2))) return st;
    TTS_HIP(hipMemsetAsync(t->tr_gran, 0, sizeof(unsigned long long) * (tres_granules() + 2), s));
    t->res_ticks = (long long)rate_khz * 50;  // 50 ms per hand-off wait
    // fault injection for the timeout fallback test (TTS_DEC_WAIT_TICKS wall-clock ticks)
    if (const char* tk = getenv("TTS_DEC_WAIT_TICKS"); tk && tk[0]) t->res_ticks = std::max(1LL, atoll(tk));
    t->resident = true;
    return TTS_OK;
}

#undef GET

}  // namespace

extern "C" {

void tts_tacotron_destroy(tts_tacotron* t) {
    if (!t) return;
    if (t->stream) (void)hipStreamSynchronize(t->stream);
    for (auto& kv : t->graphs)
        for (auto* x : {kv.second.step[0], kv.second.step[1], kv.second.chunk})
            if (x) (void)hipGraphExecDestroy(x);
    for (void* p : t->allocs) (void)hipFree(p);
    for (Buf* b : {&t->bank, &t->p0, &t->y, &t->hwa, &t->hwb, &t->xi, &t->seq_out, &t->pre_a, &t->pre_b, &t->g0, &t->g1,
                   &t->gxi, &t->gh, &t->gst_out, &t->spk_rows})
        if (b->p) (void)hipFree(b->p);
    if (t->host_flags) (void)hipHostFree(t->host_flags);
    for (hipEvent_t e : {t->ev_in, t->ev_out, t->ev_t0, t->ev_t1})
        if (e) (void)hipEventDestroy(e);
    if (t->stream) (void)hipStreamDestroy(t->stream);
    delete t;
}

tts_status tts_tacotron_create(const tts_tacotron_config* cfg, const tts_tensor* tensors, int n_tensors, void* stream,
                               tts_tacotron** out) {
    TTS_CHECK(cfg && out && (tensors || n_tensors == 0), TTS_ERR_INVALID, "null argument");
    TTS_CHECK(cfg->r >= 1 && cfg->r <= 8, TTS_ERR_INVALID, "r must be in [1, 8]");
    const int ms = cfg->memory_size > 0 ? cfg->memory_size : cfg->r;
    TTS_CHECK(ms == cfg->r, TTS_ERR_UNSUPPORTED, "memory_size must equal r (the configs' memory queue)");
    TTS_CHECK(cfg->max_batch >= 1 && cfg->max_batch <= 64, TTS_ERR_UNSUPPORTED, "max_batch must be in [1, 64]");
    TTS_CHECK(cfg->max_len >= 1 && cfg->max_len <= (cfg->location_attn ? 512 : 1024), TTS_ERR_UNSUPPORTED,
              "max_len must be in [1, 1024] (512 with location attention)");
    TTS_CHECK(cfg->max_steps >= 1, TTS_ERR_INVALID, "max_steps must be >= 1");
    TTS_CHECK(cfg->attn_norm == 0 || cfg->attn_norm == 1, TTS_ERR_INVALID, "Unknown value for attention norm type");
    TTS_CHECK(!cfg->trans_agent || cfg->forward_attn, TTS_ERR_INVALID, "trans_agent requires forward_attn");
    auto* t = new tts_tacotron();
    t->cfg = *cfg;
    t->cfg.memory_size = ms;
    t->nmel = 80 * cfg->r;
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto fail = [&](tts_status code) {
        tts_tacotron_destroy(t);
        return code;
    };
    if (hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&t->ev_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&t->ev_out, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&t->ev_t0, hipEventReleaseToDevice) != hipSuccess ||
        hipEventCreateWithFlags(&t->ev_t1, hipEventReleaseToDevice) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&t->host_flags), 4 * sizeof(int)) != hipSuccess) {
        set_error("stream/event creation failed");
        return fail(TTS_ERR_HIP);
    }
    WeightMap wm;
    for (int i = 0; i < n_tensors; ++i) wm.m[tensors[i].key] = {tensors[i].data, tensors[i].numel};
    tts_status st = fold_prenet_bn(t, wm, s);
    if (!st) st = create_weights(t, wm, s);
    if (!st) st = create_workspace(t, s);
    if (!st) st = create_resident(t, wm, s);
    if (!st && hipStreamSynchronize(s) != hipSuccess) {
        set_error("weight repacking failed");
        st = TTS_ERR_HIP;
    }
    if (st) return fail(st);
    *out = t;
    return TTS_OK;
}

tts_status tts_tacotron_encode(tts_tacotron* t, const int32_t* ids, const int32_t* lens, int B, int Lmax,
                               const int32_t* speaker_ids, const float* style_mel, int style_frames, float* out,
                               void* stream) {
    TTS_CHECK(t && ids && lens && out, TTS_ERR_INVALID, "null argument");
    TTS_CHECK(B >= 1 && B <= t->Bcap && Lmax >= 1 && Lmax <= t->Lcap, TTS_ERR_INVALID,
              "batch / length exceeds capacity");
    TTS_CHECK(!style_mel || (t->cfg.gst && style_frames >= 1), TTS_ERR_INVALID,
              "style_mel needs a TacotronGST model and style_frames >= 1");
    int frames = 0;
    for (int b = 0; b < B; ++b) {
        TTS_CHECK(lens[b] >= 1 && lens[b] <= Lmax, TTS_ERR_INVALID, "length out of range [1, Lmax]");
        frames += lens[b];
        if (speaker_ids && t->spk)
            TTS_CHECK(speaker_ids[b] >= 0 && speaker_ids[b] < t->cfg.num_speakers, TTS_ERR_INVALID,
                      "speaker id out of range");
    }
    hipStream_t cs = static_cast<hipStream_t>(stream);
    hipStream_t s = t->stream;
    TTS_HIP(hipEventRecord(t->ev_in, cs));
    TTS_HIP(hipStreamWaitEvent(s, t->ev_in, 0));
    const size_t BL = (size_t)B * Lmax;
    tts_status st;
    if ((st = grow(t, t->pre_a, BL * 256)) || (st = grow(t, t->pre_b, BL * 128)) || (st = grow(t, t->seq_out, BL * 256)) ||
        (st = grow(t, t->spk_rows, (size_t)B * 256)))
        return st;
    TTS_HIP(hipMemcpyAsync(t->ids, ids, sizeof(int) * BL, hipMemcpyDeviceToDevice, s));
    TTS_HIP(hipMemcpyAsync(t->T, lens, sizeof(int) * B, hipMemcpyHostToDevice, s));
    const float* add1 = nullptr;
    const float* add2 = nullptr;
    if (speaker_ids && t->spk) {  // _add_speaker_embedding (models/tacotrongst.py:81-90)
        TTS_HIP(hipMemcpyAsync(t->spk_ids, speaker_ids, sizeof(int) * B, hipMemcpyHostToDevice, s));
        TTS_HIP(launch_gather_rows(t->spk, t->spk_ids, 256, t->spk_rows.p, B, s));
        add1 = t->spk_rows.p;
    }
    if (style_mel) {
        if ((st = run_gst(t, style_mel, style_frames, B, s))) return st;
        add2 = t->gst_out.p;
    }
    // embedding gather + prenet layer 1 (+ ReLU), layer 2 (+ ReLU); dropout off in eval
    ConvArgs a{};
    a.ids = t->ids;
    a.table = t->emb;
    a.out = t->pre_a.p;
    a.W = t->Wep0;
    a.shift = t->bep0;
    a.T = t->T;
    a.Tmax = Lmax;
    a.Cin = 256;
    a.Cout = 256;
    a.co_pad = 256;
    a.act = CONV_RELU;
    TTS_HIP(conv_launch(a, 1, B, frames, s));
    a = ConvArgs{};
    a.in = t->pre_a.p;
    a.out = t->pre_b.p;
    a.W = t->Wep1;
    a.shift = t->bep1;
    a.T = t->T;
    a.Tmax = Lmax;
    a.Cin = 256;
    a.Cout = 128;
    a.co_pad = 128;
    a.act = CONV_RELU;
    TTS_HIP(conv_launch(a, 1, B, frames, s));
    TTS_HIP(hipMemsetAsync(t->seq_out.p, 0, sizeof(float) * BL * 256, s));
    if ((st = run_cbhg(t, t->enc, t->pre_b.p, B, Lmax, frames, t->seq_out.p, add1, add2, s))) return st;
    TTS_HIP(hipMemcpyAsync(out, t->seq_out.p, sizeof(float) * BL * 256, hipMemcpyDeviceToDevice, s));
    TTS_HIP(hipEventRecord(t->ev_out, s));
    TTS_HIP(hipStreamWaitEvent(cs, t->ev_out, 0));
    return TTS_OK;
}

tts_status tts_tacotron_decode(tts_tacotron* t, const float* enc, const int32_t* lens, int B, int Lmax, int max_steps,
                               int steps_cap, float* mel, float* stop, float* align, int32_t* n_steps, void* stream) {
    TTS_CHECK(t && enc && lens && mel && stop && n_steps, TTS_ERR_INVALID, "null argument");
    TTS_CHECK(B >= 1 && B <= t->Bcap, TTS_ERR_INVALID, "batch exceeds decoder capacity");
    TTS_CHECK(Lmax >= 1 && Lmax <= t->Lcap, TTS_ERR_INVALID, "Lmax exceeds decoder capacity");
    TTS_CHECK(max_steps >= 1 && max_steps <= t->cfg.max_steps, TTS_ERR_INVALID, "max_steps exceeds decoder capacity");
    TTS_CHECK(steps_cap >= max_steps + 1, TTS_ERR_INVALID, "steps_cap must be >= max_steps + 1");
    TTS_CHECK(!t->cfg.forward_attn_mask || Lmax >= 2, TTS_ERR_INVALID, "forward_attn_mask needs L >= 2");
    int first = 0;  // every sentence runs at least floor(L/4) + 1 steps (t > L/4)
    for (int b = 0; b < B; ++b) {
        TTS_CHECK(lens[b] >= 1 && lens[b] <= Lmax, TTS_ERR_INVALID, "encoder length out of range [1, Lmax]");
        TTS_CHECK(!t->cfg.forward_attn_mask || lens[b] >= 2, TTS_ERR_INVALID, "forward_attn_mask needs L >= 2");
        first = std::max(first, std::min(lens[b] / 4 + 1, max_steps + 1));
    }
    hipStream_t cs = static_cast<hipStream_t>(stream);
    hipStream_t s = t->stream;
    TTS_HIP(hipEventRecord(t->ev_in, cs));
    TTS_HIP(hipStreamWaitEvent(s, t->ev_in, 0));
    TTS_HIP(hipMemcpy2DAsync(t->denc, (size_t)t->Lcap * T_DEC * 4, enc, (size_t)Lmax * T_DEC * 4, (size_t)Lmax * T_DEC * 4,
                             B, hipMemcpyDeviceToDevice, s));
    TTS_HIP(hipMemcpyAsync(t->lens, lens, sizeof(int) * B, hipMemcpyHostToDevice, s));
    TTS_HIP(launch_project_inputs(t->denc, t->W_in, B, Lmax, t->Lcap, t->Pt, s, T_DEC));
    TInitArgs ia{};
    ia.B = B; ia.Lcap = t->Lcap; ia.nmel = t->nmel; ia.lens = t->lens;
    ia.att_init = t->att_init; ia.dec_init = t->dec_init; ia.mem_init = t->mem_init;
    ia.h_att = t->h_att; ia.h1 = t->h1; ia.h2 = t->h2; ia.h_pstride = (int64_t)t->Bcap * T_DEC;
    ia.xa = t->xa; ia.mem = t->mem;
    ia.alpha = t->alpha; ia.att_w = t->att_w; ia.att_cum = t->att_cum; ia.u = t->u; ia.win_idx = t->win_idx;
    ia.nidx = t->nidx; ia.tail = t->tail; ia.flag1 = t->flag1; ia.count = t->count; ia.done = t->done;
    ia.n_steps = t->n_steps; ia.state = t->state;
    TTS_HIP(launch_tacotron_init(ia, s));
    { tts_status st = enqueue_prenet_go(t, B, s); if (st) return st; }
    int run = 0;
    t->last_resident = 0;
    if (t->resident && B <= TR_SPX * TR_GROUPS && Lmax <= TR_LMAX) {
        // one persistent launch runs every step (tacotron_resident.hip), from the state the init
        // and go-frame launches above left, into the same history buffers
        TResArgs a = t->rw;
        a.B = B; a.nmel = t->nmel; a.Lcap = t->Lcap; a.Lalign = Lmax; a.max_steps = max_steps;
        a.hist_cap = t->hist_cap;
        a.lens = t->lens; a.enc = t->denc; a.Pt = t->Pt;
        a.pre1 = t->pre1; a.h_att = t->h_att; a.h1 = t->h1; a.h2 = t->h2; a.h_pstride = (int64_t)t->Bcap * T_DEC;
        a.alpha = t->alpha;
        a.mel_hist = t->mel_hist; a.stop_hist = t->stop_hist; a.align_hist = t->align_hist;
        a.done = t->done; a.n_steps = t->n_steps;
        a.gran = t->tr_gran;
        a.status = reinterpret_cast<int*>(t->tr_gran + tres_granules());
        {
            // 18-bit tag salt: after a wrap a granule left by the launch 2^18 back could match a
            // current wait (an XCD group a smaller batch left idle), so clear them on a wrap
            bool wrapped = false;
            t->res_salt = res_next_salt(t->res_salt, &wrapped);
            if (wrapped)
                TTS_HIP(hipMemsetAsync(t->tr_gran, 0, sizeof(unsigned long long) * (tres_granules() + 2), s));
        }
        a.salt = t->res_salt;
        a.timeout_ticks = t->res_ticks;
        static const int taco_first_sleep = [] {
            const char* v = getenv("TTS_TACO_FIRST_SLEEP");
            return v ? atoi(v) : 4;  // round 6: configs[4] 1.603M -> 1.615M (tools/taco_sleep_sweep.sh)
        }();
        a.first_sleep = taco_first_sleep;
        a.prof = nullptr;
        t->last_ra = a;
        TTS_HIP(hipMemsetAsync(a.status, 0, sizeof(int), s));
        TTS_HIP(hipEventRecord(t->ev_t0, s));
        bool launched = false;
        TTS_HIP(launch_tacotron_resident(a, s, &launched));
        if (!launched) {
            // the grid cannot be co-resident on this device: nothing ran, the initial state is
            // untouched; the multi-launch path serves this handle from now on
            t->resident = false;
        } else {
            TTS_HIP(hipEventRecord(t->ev_t1, s));
            TTS_HIP(hipMemcpyAsync(t->host_flags, a.status, sizeof(int), hipMemcpyDeviceToHost, s));
            TTS_HIP(hipMemcpyAsync(n_steps, t->n_steps, sizeof(int) * B, hipMemcpyDeviceToHost, s));
            TTS_HIP(hipStreamSynchronize(s));
            const int code = t->host_flags[0];
            if (code == 0) {
                for (int b = 0; b < B; ++b) run = std::max(run, (int)n_steps[b]);
                t->last_resident = 1;
            } else {
                // TR_STATUS_PLACEMENT: some XCD holds fewer than TR_RANKS workgroups, the kernel
                // stopped before touching any state (multi-launch from now on); otherwise a hand-off
                // wait timed out (a workgroup could not become resident beside other work) and every
                // wave drained: this batch re-runs from its initial state on the multi-launch path
                if (code == TR_STATUS_PLACEMENT) t->resident = false;
                else ++t->res_timeouts;
                TTS_HIP(launch_tacotron_init(ia, s));
                tts_status st = enqueue_prenet_go(t, B, s);
                if (st) return st;
            }
        }
    }
    if (!t->last_resident) {
    auto key = std::make_tuple(B, Lmax, max_steps);
    auto it = t->graphs.find(key);
    if (it == t->graphs.end()) {
        TGraphs g;
        tts_status st = build_graph(t, B, Lmax, max_steps, 0, 1, &g.step[0]);
        if (!st) st = build_graph(t, B, Lmax, max_steps, 1, 1, &g.step[1]);
        if (!st) st = build_graph(t, B, Lmax, max_steps, 0, TCHUNK, &g.chunk);
        if (st) return st;
        it = t->graphs.emplace(key, g).first;
    }
    const TGraphs& g = it->second;
    TTS_HIP(hipEventRecord(t->ev_t0, s));
    auto launch_steps = [&](int n) -> tts_status {
        while (n > 0) {
            if ((run & 1) == 0 && n >= TCHUNK) {
                TTS_HIP(hipGraphLaunch(g.chunk, s));
                run += TCHUNK;
                n -= TCHUNK;
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
        TTS_HIP(hipMemcpyAsync(t->host_flags, t->state + 2 * (run & 1), 2 * sizeof(int), hipMemcpyDeviceToHost, s));
        TTS_HIP(hipStreamSynchronize(s));
        if (t->host_flags[1] == 0) break;
        TTS_CHECK(run <= max_steps + 1, TTS_ERR_HIP, "decoder did not stop within max_steps + 1 (internal error)");
        st = launch_steps(TCHUNK);
        if (st) return st;
    }
    TTS_HIP(hipEventRecord(t->ev_t1, s));
    TTS_HIP(hipMemcpyAsync(n_steps, t->n_steps, sizeof(int) * B, hipMemcpyDeviceToHost, s));
    TTS_HIP(hipStreamSynchronize(s));
    }
    int nmax = 0;
    for (int b = 0; b < B; ++b) nmax = std::max(nmax, (int)n_steps[b]);
    const size_t nm = t->nmel;
    TTS_HIP(hipMemcpy2DAsync(mel, (size_t)steps_cap * nm * 4, t->mel_hist, (size_t)t->hist_cap * nm * 4,
                             (size_t)nmax * nm * 4, B, hipMemcpyDeviceToDevice, s));
    TTS_HIP(hipMemcpy2DAsync(stop, (size_t)steps_cap * 4, t->stop_hist, (size_t)t->hist_cap * 4, (size_t)nmax * 4, B,
                             hipMemcpyDeviceToDevice, s));
    if (align)
        TTS_HIP(hipMemcpy2DAsync(align, (size_t)steps_cap * Lmax * 4, t->align_hist, (size_t)t->hist_cap * Lmax * 4,
                                 (size_t)nmax * Lmax * 4, B, hipMemcpyDeviceToDevice, s));
    TTS_HIP(launch_zero_tail(mel, (int64_t)steps_cap * nm, t->n_steps, (int)nm, nmax, B, s));
    TTS_HIP(hipEventRecord(t->ev_out, s));
    TTS_HIP(hipStreamWaitEvent(cs, t->ev_out, 0));
    TTS_HIP(hipEventElapsedTime(&t->last_ms, t->ev_t0, t->ev_t1));
    t->last_steps = run;
    t->last_B = B;
    t->last_Lmax = Lmax;
    t->last_max_steps = max_steps;
    t->last_first = first;
    t->last_init = ia;
    return TTS_OK;
}

tts_status tts_tacotron_postnet(tts_tacotron* t, const float* mel, const int32_t* T, int B, int Tmax, float* linear,
                                void* stream) {
    TTS_CHECK(t && mel && T && linear && B >= 1 && Tmax >= 1, TTS_ERR_INVALID, "bad postnet arguments");
    TTS_CHECK(B <= t->Bcap, TTS_ERR_INVALID, "batch exceeds capacity");
    int frames = 0;
    for (int b = 0; b < B; ++b) {
        TTS_CHECK(T[b] >= 0 && T[b] <= Tmax, TTS_ERR_INVALID, "T[b] out of range");
        frames += T[b];
    }
    hipStream_t cs = static_cast<hipStream_t>(stream);
    hipStream_t s = t->stream;
    TTS_HIP(hipEventRecord(t->ev_in, cs));
    TTS_HIP(hipStreamWaitEvent(s, t->ev_in, 0));
    tts_status st;
    if ((st = grow(t, t->seq_out, (size_t)B * Tmax * 256))) return st;
    TTS_HIP(hipMemcpyAsync(t->T, T, sizeof(int) * B, hipMemcpyHostToDevice, s));
    if ((st = run_cbhg(t, t->post, mel, B, Tmax, frames, t->seq_out.p, nullptr, nullptr, s))) return st;
    TTS_HIP(hipMemsetAsync(linear, 0, sizeof(float) * (size_t)B * Tmax * NLIN, s));
    ConvArgs a{};
    a.in = t->seq_out.p;
    a.out = linear;
    a.W = t->W_ll;
    a.shift = t->b_ll;
    a.T = t->T;
    a.Tmax = Tmax;
    a.Cin = 256;
    a.Cout = NLIN;
    a.co_pad = conv_co_pad(NLIN);
    a.act = CONV_SIGMOID;
    TTS_HIP(conv_launch(a, 1, B, frames, s));
    TTS_HIP(hipEventRecord(t->ev_out, s));
    TTS_HIP(hipStreamWaitEvent(cs, t->ev_out, 0));
    return TTS_OK;
}

tts_status tts_tacotron_last_timing(tts_tacotron* t, float* loop_ms, int* steps_run) {
    TTS_CHECK(t && loop_ms && steps_run, TTS_ERR_INVALID, "null argument");
    *loop_ms = t->last_ms;
    *steps_run = t->last_steps;
    return TTS_OK;
}

tts_status tts_tacotron_last_path(tts_tacotron* t, int* resident) {
    TTS_CHECK(t && resident, TTS_ERR_INVALID, "null argument");
    *resident = t->last_resident;
    return TTS_OK;
}

tts_status tts_tacotron_resident_phases(tts_tacotron* t, float* us, int n) {
    TTS_CHECK(t && us && n >= 2 * TR_PHASES, TTS_ERR_INVALID, "bad arguments");
    TTS_CHECK(t->last_resident && t->last_steps > 0, TTS_ERR_INVALID,
              "tts_tacotron_resident_phases needs a previous resident tts_tacotron_decode");
    TTS_HIP(hipDeviceSynchronize());  // measurement only: nothing else on the device
    hipStream_t s = t->stream;
    long long* prof = nullptr;
    TTS_HIP(hipMalloc(&prof, sizeof(long long) * 2 * TR_PHASES));
    TTS_HIP(hipMemsetAsync(prof, 0, sizeof(long long) * 2 * TR_PHASES, s));
    TTS_HIP(launch_tacotron_init(t->last_init, s));
    tts_status st = enqueue_prenet_go(t, t->last_B, s);
    TResArgs a = t->last_ra;
    a.prof = prof;
    {
        bool wrapped = false;  // as in the decode path: clear the granules on a salt wrap
        t->res_salt = res_next_salt(t->res_salt, &wrapped);
        if (wrapped) TTS_HIP(hipMemsetAsync(t->tr_gran, 0, sizeof(unsigned long long) * (tres_granules() + 2), s));
    }
    a.salt = t->res_salt;
    if (!st) {
        TTS_HIP(hipMemsetAsync(a.status, 0, sizeof(int), s));
        bool launched = false;
        TTS_HIP(launch_tacotron_resident(a, s, &launched));
        if (!launched) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(prof);
            TTS_CHECK(false, TTS_ERR_UNSUPPORTED, "resident decoder cannot be co-resident on this device now");
        }
    }
    long long h[2 * TR_PHASES];
    TTS_HIP(hipMemcpyAsync(h, prof, sizeof(h), hipMemcpyDeviceToHost, s));
    TTS_HIP(hipMemcpyAsync(t->host_flags, a.status, sizeof(int), hipMemcpyDeviceToHost, s));
    TTS_HIP(hipStreamSynchronize(s));
    (void)hipFree(prof);
    if (st) return st;
    TTS_CHECK(t->host_flags[0] == 0, TTS_ERR_HIP, "resident decoder: a hand-off wait timed out");
    int dev = 0, rate_khz = 1;
    TTS_HIP(hipGetDevice(&dev));
    TTS_HIP(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev));
    for (int i = 0; i < 2 * TR_PHASES; ++i) us[i] = (float)(1e3 * (double)h[i] / rate_khz / t->last_steps);
    return TTS_OK;
}

tts_status tts_tacotron_profile(tts_tacotron* t, int reps, float* kernel_ms, int n_kernels) {
    TTS_CHECK(t && kernel_ms && n_kernels >= TTS_TACOTRON_STEP_KERNELS, TTS_ERR_INVALID, "bad profile arguments");
    TTS_CHECK(t->last_B > 0, TTS_ERR_INVALID, "tts_tacotron_profile needs a previous tts_tacotron_decode");
    reps = std::max(1, std::min(reps, t->last_first - 1));
    const int K = TTS_TACOTRON_STEP_KERNELS;
    hipEvent_t ev[K + 1];
    for (int i = 0; i <= K; ++i) TTS_HIP(hipEventCreate(&ev[i]));
    hipStream_t s = t->stream;
    TTS_HIP(launch_tacotron_init(t->last_init, s));
    tts_status st = enqueue_prenet_go(t, t->last_B, s);
    std::vector<double> acc(K, 0.0);
    for (int r = 0; r < reps && st == TTS_OK; ++r) {
        st = enqueue_step(t, t->last_B, t->last_Lmax, t->last_max_steps, r & 1, s, ev);
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

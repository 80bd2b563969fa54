// Postnet (layers/tacotron2.py:30-45) + residual (models/tacotron2.py:69-70): five Conv1d(k=5)
// + BatchNorm(eval) [+ tanh] layers on time-major [B][T][C] activations, per sentence at its own
// length (zero padding past T_b), as fp32 MFMA implicit GEMMs (conv1d.hip).
// Roofline: MFMA-fp32 bound, 8.68 MFLOP per frame.
#include <string>

#include <algorithm>

#include <cstdlib>
#include "conv1d.h"

using namespace tts;

struct tts_postnet {
    int n_mel = 80;
    int cin[5], cout[5], co_pad[5];
    float* W[5] = {};
    float* Wf[5] = {};  // fragment-order copies (conv_pack_frag): the small-batch conv kernel
    int wf_tap[5] = {};  // ... in the tap-major order of its Cin = 512 form (conv_pack_frag_tap)
    float* Wf16[5] = {};  // ... and its 16-channel order (conv_pack_frag_tap16) for those layers
    float* scale[5] = {};
    float* shift[5] = {};
    float* buf[2] = {};
    size_t buf_floats = 0;
    int* T = nullptr;
    int Tcap_B = 0;
    float* part = nullptr;  // split-K workspace (CONV_SPLITK_FLOATS)
};

extern "C" {

void tts_postnet_destroy(tts_postnet* p) {
    if (!p) return;
    for (int i = 0; i < 5; ++i) {
        if (p->W[i]) (void)hipFree(p->W[i]);
        if (p->Wf[i]) (void)hipFree(p->Wf[i]);
        if (p->Wf16[i]) (void)hipFree(p->Wf16[i]);
        if (p->scale[i]) (void)hipFree(p->scale[i]);
        if (p->shift[i]) (void)hipFree(p->shift[i]);
    }
    for (int i = 0; i < 2; ++i)
        if (p->buf[i]) (void)hipFree(p->buf[i]);
    if (p->part) (void)hipFree(p->part);
    if (p->T) (void)hipFree(p->T);
    delete p;
}

tts_status tts_postnet_create(const tts_tensor* tensors, int n_tensors, int n_mel, void* stream, tts_postnet** out) {
    TTS_CHECK(tensors && out && n_mel > 0 && n_mel % 16 == 0, TTS_ERR_INVALID, "bad postnet arguments");
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto* p = new tts_postnet();
    p->n_mel = n_mel;
    const int ch[6] = {n_mel, 512, 512, 512, 512, n_mel};
    auto find = [&](const std::string& key, int64_t numel) -> const float* {
        for (int i = 0; i < n_tensors; ++i)
            if (key == tensors[i].key) {
                if (tensors[i].numel != numel) { set_error("weight " + key + " has wrong size"); return nullptr; }
                return tensors[i].data;
            }
        set_error("missing weight " + key);
        return nullptr;
    };
    for (int l = 0; l < 5; ++l) {
        const std::string pre = "postnet.convolutions." + std::to_string(l) + ".net.";
        const int ci = ch[l], co = ch[l + 1];
        p->cin[l] = ci;
        p->cout[l] = co;
        p->co_pad[l] = conv_co_pad(co);
        const float* w = find(pre + "0.weight", (int64_t)co * ci * 5);
        const float* bias = find(pre + "0.bias", co);
        const float* g = find(pre + "1.weight", co);
        const float* be = find(pre + "1.bias", co);
        const float* mu = find(pre + "1.running_mean", co);
        const float* var = find(pre + "1.running_var", co);
        if (!w || !bias || !g || !be || !mu || !var) { tts_postnet_destroy(p); return TTS_ERR_INVALID; }
        const int64_t nw = (int64_t)ci * 5 * p->co_pad[l];
        if (hipMalloc(&p->W[l], nw * 4) != hipSuccess || hipMalloc(&p->Wf[l], nw * 4) != hipSuccess ||
            hipMalloc(&p->scale[l], co * 4) != hipSuccess ||
            hipMalloc(&p->shift[l], co * 4) != hipSuccess) {
            tts_postnet_destroy(p);
            set_error("hipMalloc failed");
            return TTS_ERR_NOMEM;
        }
        hipError_t e = conv_pack(w, co, ci, 5, p->W[l], s);
        p->wf_tap[l] = conv_frag_tap_ok(ci) ? 1 : 0;
        if (e == hipSuccess)
            e = p->wf_tap[l] ? conv_pack_frag_tap(p->W[l], ci, 5, p->co_pad[l], p->Wf[l], s)
                             : conv_pack_frag(p->W[l], ci * 5, p->co_pad[l], p->Wf[l], s);
        if (e == hipSuccess && p->wf_tap[l]) {
            e = hipMalloc(&p->Wf16[l], nw * 4);
            if (e == hipSuccess) e = conv_pack_frag_tap16(p->W[l], ci, 5, p->co_pad[l], p->Wf16[l], s);
        }
        if (e == hipSuccess) e = fold_bn(bias, g, be, mu, var, co, 1e-5f, p->scale[l], p->shift[l], s);
        if (e != hipSuccess) { tts_postnet_destroy(p); return hip_fail(e, "postnet pack", __FILE__, __LINE__); }
    }
    // split-K partials, then the fused reduction's ticket words (zero at rest)
    hipError_t e = hipMalloc(&p->part, CONV_SPLITK_FLOATS * sizeof(float) + CONV_TICKETS * sizeof(int));
    if (e == hipSuccess) e = hipMemsetAsync(p->part + CONV_SPLITK_FLOATS, 0, CONV_TICKETS * sizeof(int), s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) { tts_postnet_destroy(p); return hip_fail(e, "postnet pack", __FILE__, __LINE__); }
    *out = p;
    return TTS_OK;
}

tts_status tts_postnet_run(tts_postnet* p, const float* mel, const int32_t* T, int B, int Tmax, float* out,
                           void* stream) {
    return tts::postnet_run_dev(p, mel, 0, nullptr, 1, T, B, Tmax, out, static_cast<hipStream_t>(stream));
}

}  // extern "C"

namespace tts {
namespace {
__global__ void postnet_pad_kernel() {}
bool pad_kernel() {  // TTS_PAD_KERNEL=1: a trivial launch after every layer (dispatch-position diagnostic)
    static const bool on = [] {
        const char* v = getenv("TTS_PAD_KERNEL");
        return v && v[0] == '1';
    }();
    return on;
}
}  // namespace
// tts_postnet_run, optionally with the frame counts already on the device (T_dev[b] * tmul frames:
// the decoder's step counts) and the input rows mel_tmax frames apart (0 = Tmax): the synthesis
// path feeds the decoder's mel history in place, with no copy and no host-to-device transfer.
// T gives the host-side counts that size the tiles: with T_dev, an upper bound of the device counts
// (frames past T[b] are not computed; the caller redoes a sentence whose device count exceeds it).
tts_status postnet_run_dev(tts_postnet* p, const float* mel, int mel_tmax, const int* T_dev, int tmul, const int32_t* T,
                           int B, int Tmax, float* out, hipStream_t s) {
    TTS_CHECK(p && mel && T && out && B >= 1 && Tmax >= 1, TTS_ERR_INVALID, "bad postnet_run arguments");
    int frames = 0, Tlong = 1;
    for (int b = 0; b < B; ++b) {
        TTS_CHECK(T[b] >= 0 && T[b] <= Tmax, TTS_ERR_INVALID, "T[b] out of range");
        frames += T[b];
        Tlong = std::max(Tlong, (int)T[b]);
    }
    const size_t need = (size_t)B * Tmax * 512;
    if (need > p->buf_floats) {
        for (int i = 0; i < 2; ++i) {
            if (p->buf[i]) (void)hipFree(p->buf[i]);
            p->buf[i] = nullptr;
            TTS_HIP(hipMalloc(&p->buf[i], need * 4));
        }
        p->buf_floats = need;
    }
    if (B > p->Tcap_B) {
        if (p->T) (void)hipFree(p->T);
        p->T = nullptr;
        TTS_HIP(hipMalloc(&p->T, B * sizeof(int)));
        p->Tcap_B = B;
    }
    if (!T_dev) TTS_HIP(hipMemcpyAsync(p->T, T, B * sizeof(int), hipMemcpyHostToDevice, s));
    const float* in = mel;
    for (int l = 0; l < 5; ++l) {
        ConvArgs a{};
        a.in = in;
        a.out = l == 4 ? out : p->buf[l & 1];
        a.W = p->W[l];
        a.Wf = p->Wf[l];
        a.wf_tap = p->wf_tap[l];
        a.Wf16 = p->Wf16[l];
        a.scale = p->scale[l];
        a.shift = p->shift[l];
        a.resid = l == 4 ? mel : nullptr;
        a.T = T_dev ? T_dev : p->T;
        a.tmul = T_dev ? tmul : 1;
        a.Tmax = Tmax;
        a.in_tmax = l == 0 ? mel_tmax : 0;
        a.res_tmax = l == 4 ? mel_tmax : 0;
        a.Cin = p->cin[l];
        a.Cout = p->cout[l];
        a.co_pad = p->co_pad[l];
        a.act = l < 4 ? CONV_TANH : CONV_NONE;
        a.part = p->part;
        a.tickets = reinterpret_cast<int*>(p->part + CONV_SPLITK_FLOATS);
        a.Ttile = Tlong;
        TTS_HIP(conv_launch(a, 5, B, frames, s));
        if (pad_kernel()) hipLaunchKernelGGL(postnet_pad_kernel, dim3(1), dim3(64), 0, s);  // measurement only
        in = a.out;
    }
    return TTS_OK;
}
}  // namespace tts

// Microbenchmark of the decoder's attention launch (the library's attention.hip compiled in) as
// a dependent chain in a hipGraph, batch 1, L = 100, forward attention + mask + sigmoid norm
// (the bench configuration).  Build with -DATT_BISECT=k on a patched copy to price sections.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../your-voice-tts_amd/csrc \
//         -o attn_chain attn_chain.hip ../../your-voice-tts_amd/csrc/attention.hip
#include <cstdio>
#include <functional>
#include <vector>

#include "decoder.h"

using namespace tts;

static float time_chain(hipStream_t s, int n, const std::function<void(int)>& launch) {
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < n; ++i) launch(i);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int w = 0; w < 3; ++w) (void)hipGraphLaunch(ge, s);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, s);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) (void)hipGraphLaunch(ge, s);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    return 1000.f * ms / (reps * n);
}

template <typename T>
static T* dalloc(size_t n, float fill = 0.f) {
    void* p = nullptr;
    if (hipMalloc(&p, n * sizeof(T) + 64) != hipSuccess) return nullptr;
    std::vector<T> h(n + 16, (T)fill);
    (void)hipMemcpy(p, h.data(), (n + 16) * sizeof(T), hipMemcpyHostToDevice);
    return static_cast<T*>(p);
}

int main(int argc, char** argv) {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    const int B = 1, L = argc > 1 ? atoi(argv[1]) : 100, Lc = 128;
    AttnArgs a{};
    a.attn_norm = 1;
    a.forward_attn = 1;
    a.forward_attn_mask = 1;
    a.Lcap = Lc;
    a.B = B;
    a.v = dalloc<float>(ADIM, 0.01f);
    a.v_b = dalloc<float>(1);
    a.ta_w = dalloc<float>(1536);
    a.ta_b = dalloc<float>(1);
    a.q = dalloc<float>(B * ADIM, 0.1f);
    a.Pt = dalloc<float>(B * ADIM * Lc, 0.05f);
    a.enc = dalloc<float>(B * Lc * ENC, 0.02f);
    std::vector<int> hl(B, L);
    int* lens = dalloc<int>(B);
    (void)hipMemcpy(lens, hl.data(), B * sizeof(int), hipMemcpyHostToDevice);
    a.lens = lens;
    a.h_att = dalloc<float>(B * HATT);
    a.epart = dalloc<float>((size_t)B * QE_TILES * Lc, 0.01f);
    a.alpha = dalloc<float>(B * Lc, 0.01f);
    a.att_w = dalloc<float>(B * Lc);
    a.att_cum = dalloc<float>(B * Lc);
    a.u = dalloc<float>(B, 0.5f);
    a.win_idx = dalloc<int>(B);
    int* nidx = dalloc<int>(B);
    int one = 1;
    (void)hipMemcpy(nidx, &one, sizeof(int), hipMemcpyHostToDevice);
    a.nidx = nidx;
    a.tail = dalloc<float>(B);
    a.ctx = dalloc<float>(B * XA);
    a.align_hist = dalloc<float>((size_t)B * 4 * Lc);
    a.align_ldb = 4 * Lc;
    a.Lalign = L;
    a.hist_cap = 4;
    int* st = dalloc<int>(4);
    int stv[4] = {0, 1, 0, 1};
    (void)hipMemcpy(st, stv, sizeof(stv), hipMemcpyHostToDevice);
    a.step = st;
    a.done = dalloc<int>(B);
    (void)attention_prepare(Lc, 0);
    const float us = time_chain(s, 200, [&](int) { (void)launch_attention(a, s); });
    printf("attention B=%d L=%d: %7.2f us/launch\n", B, L, us);
    QEArgs qa{};
    qa.Wq = dalloc<float>((size_t)ADIM * HATT, 0.001f);
    qa.h = a.h_att;
    qa.v = a.v;
    qa.Pt = a.Pt;
    qa.lens = lens;
    qa.Lcap = Lc;
    qa.energies = 1;
    qa.q = const_cast<float*>(a.q);
    qa.epart = const_cast<float*>(a.epart);
    qa.step = st;
    const float uq = time_chain(s, 200, [&](int) { (void)launch_query_energy(qa, B, s); });
    printf("query+energy B=%d L=%d: %7.2f us/launch\n", B, L, uq);
    const float up = time_chain(s, 200, [&](int k) {
        if (k & 1) (void)launch_attention(a, s); else (void)launch_query_energy(qa, B, s);
    });
    printf("pair: %7.2f us per query+attention\n", 2 * up);
    return 0;
}

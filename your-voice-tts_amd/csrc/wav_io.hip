// Synthesizer.tts's waveform join and AudioProcessor.save_wav's int16 conversion on the device
// (server/synthesizer.py:157-161, utils/audio.py:56-58):
//   wavs = [s_0, 10000 zeros, s_1, 10000 zeros, ...];  pcm = (wavs * (32767 / max(0.01, max|wavs|))).astype(int16)
// The reference builds that as a Python list of floats (~80 ms per 3000-frame sentence here) and
// converts it with numpy; the sentences are already in HBM, so the join is two launches: a max-abs
// reduction over every sentence's samples (|y| as IEEE bits: order-free, the same maximum numpy
// finds) and one pass that writes the int16 samples with the gaps in place.  The arithmetic is
// numpy's: the scale is one float64 division, each sample one float64 product truncated toward
// zero (the C conversion astype(int16) performs), so the bytes equal the reference's.
#include "common.h"

namespace tts {
namespace {

constexpr int PCM_THREADS = 256;
constexpr int PCM_PER = 8;  // samples per thread

struct PcmArgs {
    const double* wav;
    int64_t pitch;
    const int64_t* start;   // [B + 1] output offset of sentence b (its samples, then `gap` zeros)
    int B;
    int gap;
    unsigned long long* peak;  // [1] max |y| as IEEE bits (non-negative doubles order like their bits)
    double fixed_peak;         // >= 0: the peak to use (a sharded request's all-ranks maximum)
    int16_t* out;
};

__device__ __forceinline__ int find_sentence(const int64_t* start, int B, int64_t i) {
    int lo = 0, up = B - 1;
    while (lo < up) {
        const int mid = (lo + up + 1) >> 1;
        if (start[mid] <= i) lo = mid;
        else up = mid - 1;
    }
    return lo;
}

__global__ __launch_bounds__(PCM_THREADS) void pcm_peak_kernel(const PcmArgs a) {
    const int b = blockIdx.y;
    const int64_t n = a.start[b + 1] - a.start[b] - a.gap;
    const double* y = a.wav + (int64_t)b * a.pitch;
    double m = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * PCM_THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * PCM_THREADS)
        m = fmax(m, fabs(y[i]));
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
    __shared__ double wm[PCM_THREADS / 64];
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < PCM_THREADS / 64; ++w) m = fmax(m, wm[w]);
        atomicMax(a.peak, (unsigned long long)__double_as_longlong(m));
    }
}

__global__ __launch_bounds__(PCM_THREADS) void pcm_write_kernel(const PcmArgs a) {
    const double peak = a.fixed_peak >= 0.0 ? a.fixed_peak : __longlong_as_double((long long)*a.peak);
    const double scale = 32767.0 / fmax(0.01, peak);
    const int64_t total = a.start[a.B];
    const int64_t i0 = ((int64_t)blockIdx.x * PCM_THREADS + threadIdx.x) * PCM_PER;
    if (i0 >= total) return;
    int b = find_sentence(a.start, a.B, i0);
#pragma unroll
    for (int k = 0; k < PCM_PER; ++k) {
        const int64_t i = i0 + k;
        if (i >= total) break;
        while (b + 1 < a.B && i >= a.start[b + 1]) ++b;
        const int64_t j = i - a.start[b];
        const int64_t n = a.start[b + 1] - a.start[b] - a.gap;
        a.out[i] = j < n ? (int16_t)(int)(a.wav[(int64_t)b * a.pitch + j] * scale) : (int16_t)0;
    }
}

}  // namespace

// start: [dev] B + 1 output offsets (start[b + 1] - start[b] = n_b + gap); peak_bits: [dev] one
// word, overwritten (peak >= 0: that peak is used, else max |y| over the request)
hipError_t pcm16_join(const double* wav, int64_t pitch, const int64_t* start_dev, int64_t total, int B, int gap,
                      double peak, unsigned long long* peak_bits, int16_t* out, hipStream_t s) {
    PcmArgs a{wav, pitch, start_dev, B, gap, peak_bits, peak, out};
    hipError_t e;
    if (peak < 0.0) {
        if ((e = hipMemsetAsync(peak_bits, 0, sizeof(*peak_bits), s)) != hipSuccess) return e;
        hipLaunchKernelGGL(pcm_peak_kernel, dim3(64, B), dim3(PCM_THREADS), 0, s, a);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    const int64_t per_block = (int64_t)PCM_THREADS * PCM_PER;
    if (total > 0)
        hipLaunchKernelGGL(pcm_write_kernel, dim3((unsigned)((total + per_block - 1) / per_block)), dim3(PCM_THREADS), 0, s, a);
    return hipGetLastError();
}

}  // namespace tts

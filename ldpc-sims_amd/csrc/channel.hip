// channel.hip — OFDM front end on device: the reference's transmit_symbols / demodulate_signal.
//
//   modulate_bits      ofdm/ofdm_functions.py:17-22  QPSK: s = ((1-2 b0) + j (1-2 b1)) / sqrt(2), bits in pairs
//                      16-QAM (new, not in the reference; Gray per dimension):
//                      re = (1-2 b0)(3-2 b1)/sqrt(10), im = (1-2 b2)(3-2 b3)/sqrt(10)
//   transmit_symbols   :25-35  blocks of N = ofdm_size symbols -> unitary IDFT (DFT(N).conj().T @ s)
//                      + complex AWGN (N(0, 1/sqrt(snr)) + j N(0, 1/sqrt(snr))) / sqrt(2)
//   demodulate_signal  :63-78  unitary DFT (DFT(N) @ r); noise_power = 0.5/snr per real dimension;
//                      LLR = log P(1)/P(0): QPSK ((y - a)^2 - (y + a)^2) / (2 np), a = 1/sqrt(2);
//                      16-QAM: exact log-sum-exp over the two levels of each bit value per dimension.
// One workgroup handles 256/N OFDM blocks (N <= 256): symbols staged in LDS, each thread computes one
// output sample/subcarrier as an N-term complex dot product against an exact twiddle table.
#include "common.h"

namespace ldpc {

constexpr float kInvSqrt2 = 0.70710678118654752f;
constexpr float kInvSqrt10 = 0.31622776601683794f;

__device__ __forceinline__ float2 map_symbol(const uint8_t* b, int bps) {
    if (bps == 2) return make_float2((1.0f - 2.0f * b[0]) * kInvSqrt2, (1.0f - 2.0f * b[1]) * kInvSqrt2);
    return make_float2((1.0f - 2.0f * b[0]) * (3.0f - 2.0f * b[1]) * kInvSqrt10,
                       (1.0f - 2.0f * b[2]) * (3.0f - 2.0f * b[3]) * kInvSqrt10);
}

// twiddle exp(sign * j 2 pi q / N) for q in [0, N): sincospi in double, rounded once
__device__ __forceinline__ void twiddles(float2* tw, int N, float sgn) {
    for (int q = threadIdx.x; q < N; q += blockDim.x) {
        double s, c;
        sincospi(2.0 * q / N, &s, &c);
        tw[q] = make_float2((float)c, (float)(sgn * s));
    }
}

__global__ __launch_bounds__(256) void k_ofdm_tx(const uint8_t* __restrict__ bits, int64_t nsym, int N, int bps,
                                                 float nstd, uint64_t seed, int64_t sym0, float2* __restrict__ rx,
                                                 float2* __restrict__ tx) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float2* tw = (float2*)smem;           // [N]
    float2* sy = tw + N;                  // [blockDim]
    twiddles(tw, N, +1.0f);
    const int per = blockDim.x / N;       // OFDM blocks per workgroup
    const int lb = threadIdx.x / N, k = threadIdx.x % N;
    const int64_t blk = (int64_t)blockIdx.x * per + lb;
    const int64_t i = blk * N + k;        // symbol / sample index in the stream
    const bool ok = lb < per && i < nsym;
    if (ok) sy[threadIdx.x] = map_symbol(bits + i * bps, bps);
    __syncthreads();
    if (!ok) return;
    const float2* s = sy + lb * N;
    float re = 0.0f, im = 0.0f;
    for (int q = 0; q < N; ++q) {  // x[t=k] = sum_q s[q] e^{+j 2 pi q t / N} / sqrt(N)
        const float2 w = tw[(q * k) % N];
        re += s[q].x * w.x - s[q].y * w.y;
        im += s[q].x * w.y + s[q].y * w.x;
    }
    const float sc = rsqrtf((float)N);
    re *= sc;
    im *= sc;
    if (tx) tx[i] = make_float2(re, im);
    uint32_t r[4];
    Philox::gen((uint64_t)(sym0 + i), seed ^ 0xD1B54A32D192ED03ull, r);
    const float u1 = ((float)r[0] + 1.0f) * 2.3283064365386963e-10f;
    const float u2 = (float)r[1] * 2.3283064365386963e-10f;
    const float rad = sqrtf(-2.0f * logf(u1));
    float sn, cs;
    sincospif(2.0f * u2, &sn, &cs);
    rx[i] = make_float2(re + nstd * rad * cs, im + nstd * rad * sn);
}

// exact LLR log P(b=1)/P(b=0) of one 16-QAM dimension (Gray levels (1-2ba)(3-2bb)/sqrt(10))
__device__ __forceinline__ void llr_16qam_dim(float y, float inv2np, float* la, float* lb) {
    // metric of level v: -(y - v)^2 / (2 np)
    const float l3 = 3.0f * kInvSqrt10, l1 = kInvSqrt10;
    const float m00 = -(y - l3) * (y - l3) * inv2np;   // ba=0, bb=0: +3
    const float m01 = -(y - l1) * (y - l1) * inv2np;   // ba=0, bb=1: +1
    const float m11 = -(y + l1) * (y + l1) * inv2np;   // ba=1, bb=1: -1
    const float m10 = -(y + l3) * (y + l3) * inv2np;   // ba=1, bb=0: -3
    auto lse = [](float a, float b) { const float mx = fmaxf(a, b); return mx + log1pf(expf(-fabsf(a - b))); };
    *la = lse(m11, m10) - lse(m00, m01);
    *lb = lse(m01, m11) - lse(m00, m10);
}

__global__ __launch_bounds__(256) void k_ofdm_demod(const float2* __restrict__ rx, int64_t nsym, int N, int bps,
                                                    float snr, float* __restrict__ llr, float2* __restrict__ sym) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float2* tw = (float2*)smem;
    float2* r = tw + N;
    twiddles(tw, N, -1.0f);
    const int per = blockDim.x / N;
    const int lb = threadIdx.x / N, k = threadIdx.x % N;
    const int64_t blk = (int64_t)blockIdx.x * per + lb;
    const int64_t i = blk * N + k;
    const bool ok = lb < per && i < nsym;
    if (ok) r[threadIdx.x] = rx[i];
    __syncthreads();
    if (!ok) return;
    const float2* x = r + lb * N;
    float re = 0.0f, im = 0.0f;
    for (int t = 0; t < N; ++t) {  // S[k] = sum_t r[t] e^{-j 2 pi k t / N} / sqrt(N)
        const float2 w = tw[(k * t) % N];
        re += x[t].x * w.x - x[t].y * w.y;
        im += x[t].x * w.y + x[t].y * w.x;
    }
    const float sc = rsqrtf((float)N);
    re *= sc;
    im *= sc;
    if (sym) sym[i] = make_float2(re, im);
    const float np = 0.5f / snr;  // ofdm_functions.py:70
    if (bps == 2) {
        const float a = kInvSqrt2;
        llr[i * 2 + 0] = ((re - a) * (re - a) - (re + a) * (re + a)) / (2.0f * np);
        llr[i * 2 + 1] = ((im - a) * (im - a) - (im + a) * (im + a)) / (2.0f * np);
    } else {
        const float inv2np = 1.0f / (2.0f * np);
        llr_16qam_dim(re, inv2np, &llr[i * 4 + 0], &llr[i * 4 + 1]);
        llr_16qam_dim(im, inv2np, &llr[i * 4 + 2], &llr[i * 4 + 3]);
    }
}

// ---- ADC quantizer (quantizer / gen_qdata, ofdm_functions.py:37-51,118-128) ----
// AGC: sigma = np.std(rx) over the complex stream = sqrt(mean |x - mean x|^2), in fp64, deterministic
// (fixed grid of partial sums reduced in a fixed order by one workgroup).
constexpr int kMomBlocks = 512;

__global__ __launch_bounds__(256) void k_moments(const float2* __restrict__ x, int64_t n, double* __restrict__ part) {
    __shared__ double sh[3][256];
    double sr = 0.0, si = 0.0, sq = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float2 v = x[i];
        sr += v.x;
        si += v.y;
        sq += (double)v.x * v.x + (double)v.y * v.y;
    }
    sh[0][threadIdx.x] = sr;
    sh[1][threadIdx.x] = si;
    sh[2][threadIdx.x] = sq;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int c = 0; c < 3; ++c) sh[c][threadIdx.x] += sh[c][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x < 3) part[blockIdx.x * 3 + threadIdx.x] = sh[threadIdx.x][0];
}

// part[kMomBlocks][3] -> part[0] = clip = sigma * clip_ratio
__global__ __launch_bounds__(256) void k_agc_clip(double* __restrict__ part, int64_t n, double clip_ratio) {
    __shared__ double sh[3][256];
    for (int c = 0; c < 3; ++c) {
        double a = 0.0;
        for (int b = threadIdx.x; b < kMomBlocks; b += 256) a += part[b * 3 + c];
        sh[c][threadIdx.x] = a;
    }
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int c = 0; c < 3; ++c) sh[c][threadIdx.x] += sh[c][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double mr = sh[0][0] / n, mi = sh[1][0] / n;
        const double var = fmax(sh[2][0] / n - (mr * mr + mi * mi), 0.0);
        part[0] = sqrt(var) * clip_ratio;
    }
}

// q = clip(step * floor(x / step + .5), -(L/2) step + 1, (L/2) step - 1), step = 2 clip / (L - 1), in fp64
// exactly as written (the +-1 in the bounds mixes units, ofdm_functions.py:44-45; lo > hi gives hi, as
// np.clip does).  clip comes from the device (AGC) when clip_dev != nullptr.
__global__ __launch_bounds__(256) void k_adc(const float2* __restrict__ x, int64_t n, int nbits, double clip_host,
                                             const double* __restrict__ clip_dev, float2* __restrict__ q) {
    const double clip = clip_dev ? clip_dev[0] : clip_host;
    const double L = (double)(1ll << nbits);
    const double step = 2.0 * clip / (L - 1.0);
    const double lo = -(L / 2.0) * step + 1.0, hi = (L / 2.0) * step - 1.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float2 v = x[i];
        const double re = fmin(fmax(step * floor((double)v.x / step + 0.5), lo), hi);
        const double im = fmin(fmax(step * floor((double)v.y / step + 0.5), lo), hi);
        q[i] = make_float2((float)re, (float)im);
    }
}

}  // namespace ldpc

using namespace ldpc;

extern "C" {

int ldpc_ofdm_tx(const uint8_t* bits, int64_t nsym, int32_t ofdm_size, int32_t bits_per_symbol, float snr,
                 uint64_t seed, int64_t sym0, float* rx_out, float* tx_out, void* stream) {
    if (!bits || !rx_out || nsym < 0 || ofdm_size <= 0 || ofdm_size > 256 || (bits_per_symbol != 2 && bits_per_symbol != 4) ||
        !(snr > 0.0f) || sym0 < 0)
        return set_error(LDPC_EINVAL, "bad ofdm_tx arguments");
    if (nsym % ofdm_size) return set_error(LDPC_EINVAL, "nsym (%lld) must be a multiple of ofdm_size (%d)", (long long)nsym, ofdm_size);
    if (nsym == 0) return LDPC_OK;
    const int per = 256 / ofdm_size;
    const int64_t blocks = (nsym / ofdm_size + per - 1) / per;
    const float nstd = 1.0f / sqrtf(snr) / sqrtf(2.0f);  // (N(0,1/sqrt(snr)) + j N(0,1/sqrt(snr)))/sqrt(2)
    const size_t lds = sizeof(float2) * (ofdm_size + per * ofdm_size);
    k_ofdm_tx<<<(unsigned)blocks, per * ofdm_size, lds, (hipStream_t)stream>>>(bits, nsym, ofdm_size, bits_per_symbol, nstd,
                                                                              seed, sym0, (float2*)rx_out, (float2*)tx_out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(LDPC_EHIP, "ofdm_tx: %s", hipGetErrorString(e));
    return LDPC_OK;
}

int ldpc_ofdm_demod(const float* rx, int64_t nsym, int32_t ofdm_size, int32_t bits_per_symbol, float snr, float* llr_out,
                    float* sym_out, void* stream) {
    if (!rx || !llr_out || nsym < 0 || ofdm_size <= 0 || ofdm_size > 256 || (bits_per_symbol != 2 && bits_per_symbol != 4) ||
        !(snr > 0.0f))
        return set_error(LDPC_EINVAL, "bad ofdm_demod arguments");
    if (nsym % ofdm_size) return set_error(LDPC_EINVAL, "nsym (%lld) must be a multiple of ofdm_size (%d)", (long long)nsym, ofdm_size);
    if (nsym == 0) return LDPC_OK;
    const int per = 256 / ofdm_size;
    const int64_t blocks = (nsym / ofdm_size + per - 1) / per;
    const size_t lds = sizeof(float2) * (ofdm_size + per * ofdm_size);
    k_ofdm_demod<<<(unsigned)blocks, per * ofdm_size, lds, (hipStream_t)stream>>>((const float2*)rx, nsym, ofdm_size,
                                                                                 bits_per_symbol, snr, llr_out, (float2*)sym_out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(LDPC_EHIP, "ofdm_demod: %s", hipGetErrorString(e));
    return LDPC_OK;
}

int ldpc_adc_quantize(const float* rx, int64_t nsym, int32_t num_bits, double clip_ratio, double clip_value,
                      float* q_out, double* clip_out, void* stream) {
    if (!rx || !q_out || nsym < 0 || num_bits < 1 || num_bits > 24 || (clip_ratio > 0.0) == (clip_value > 0.0))
        return set_error(LDPC_EINVAL, "bad adc_quantize arguments (exactly one of clip_ratio / clip_value must be > 0)");
    if (nsym == 0) return LDPC_OK;
    hipStream_t st = (hipStream_t)stream;
    double* part = nullptr;
    if (clip_ratio > 0.0) {
        if (hipMallocAsync((void**)&part, sizeof(double) * 3 * kMomBlocks, st) != hipSuccess)
            return set_error(LDPC_ENOMEM, "adc_quantize: scratch allocation failed");
        k_moments<<<kMomBlocks, 256, 0, st>>>((const float2*)rx, nsym, part);
        k_agc_clip<<<1, 256, 0, st>>>(part, nsym, clip_ratio);
        if (clip_out) (void)hipMemcpyAsync(clip_out, part, sizeof(double), hipMemcpyDeviceToDevice, st);
    }
    const int64_t want = (nsym + 255) / 256;
    const unsigned grid = (unsigned)(want < 8192 ? want : 8192);
    k_adc<<<grid, 256, 0, st>>>((const float2*)rx, nsym, num_bits, clip_value, part, (float2*)q_out);
    if (part) (void)hipFreeAsync(part, st);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(LDPC_EHIP, "adc_quantize: %s", hipGetErrorString(e));
    return LDPC_OK;
}

}  // extern "C"

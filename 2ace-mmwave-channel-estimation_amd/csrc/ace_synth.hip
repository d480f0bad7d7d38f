// Synthetic traces on the device, with the semantics of the reference generators:
//   codebook : Generate_Sensing_Matrix.m:85-122 ('Random_Phase_State'):
//              FW = exp(1j*2*pi*k/4)/sqrt(Nt*Nr), k ~ U{0..3} i.i.d. per entry
//   channel  : Generate_Channel.m:64-164 (on_grid = 0, L paths, Rician_K = 0 for L > 1):
//              H = sqrt(Nt*Nr) * ARx * diag(h) * ATx', AoD/AoA ~ U(-95/2, 95/2) deg
//              (Searching_Area = 95, channel_recovery_ADMM_v2_simulation_A2only.m:52),
//              h ~ CN(0,1) normalised to unit norm, vecH = vec(H) column-major
//   measure  : Generate_Measurement.m:67-136: B = |FW vecH + w|, w ~ CN(0, 10^(-SNR/10))
//   scaling  : B, X0, vecH divided by ||B|| (the normalisation InferADMM's inputs get,
//              inferLowRankV4_multi.m:32-38)
// The RNG is counter based (splitmix64 of seed/stream/counter), so the integer
// streams (codebook phase states) are bit-identical to ace_amd/synth.py.
#include "ace_common.hpp"

namespace ace {

__host__ __device__ inline uint64_t sm64(uint64_t seed, uint64_t stream, uint64_t ctr) {
    uint64_t z = (seed ^ (stream * 0xD1B54A32D192ED03ULL)) + (ctr + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__device__ inline double u01(uint64_t seed, uint64_t stream, uint64_t ctr) {
    return (double)(sm64(seed, stream, ctr) >> 11) * (1.0 / 9007199254740992.0);
}
// standard normal pair (Box-Muller) from counters 2c, 2c+1
__device__ inline d2 nrm2(uint64_t seed, uint64_t stream, uint64_t c) {
    const double u1 = u01(seed, stream, 2 * c), u2 = u01(seed, stream, 2 * c + 1);
    const double r = sqrt(-2.0 * log(1.0 - u1));
    double s, co;
    sincos(2.0 * M_PI * u2, &s, &co);
    return make_double2(r * co, r * s);
}

// stream ids: kind + 16 * (realisation + 1) for per-realisation streams, kind for shared ones
enum { ST_CODEBOOK = 1, ST_ANGLES = 2, ST_GAINS = 3, ST_NOISE = 4, ST_X0 = 5 };
__device__ inline uint64_t stream_id(int kind, long long real) {
    return (uint64_t)kind + (real < 0 ? 0ULL : 16ULL * (uint64_t)(real + 1));
}

namespace {
__global__ void codebook_kernel(uint64_t seed, long long first, int count, int m, int n, double* Ap) {
    const long long total = (long long)count * m * n;
    const double s = 1.0 / sqrt((double)n);
    d2* A = reinterpret_cast<d2*>(Ap);
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        const long long c = e / ((long long)m * n), w = e - c * (long long)m * n;
        const long long real = first < 0 ? -1 : first + c;
        const int k = (int)(sm64(seed, stream_id(ST_CODEBOOK, real), (uint64_t)w) >> 62);
        // j^k / sqrt(n)
        const double re = (k == 0) ? s : (k == 2 ? -s : 0.0);
        const double im = (k == 1) ? s : (k == 3 ? -s : 0.0);
        A[e] = make_double2(re, im);
    }
}

// one work-group per realisation
__global__ __launch_bounds__(256) void channel_kernel(uint64_t seed, long long first, int m, int tx, int rx, int L,
                                                      double sigma2, double x0_noise, const double* Ap, int a_shared,
                                                      double* vecHp, double* Bp, double* X0p, double lam_d) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    d2* h = reinterpret_cast<d2*>(smem);                 // [n]
    double* sd = reinterpret_cast<double*>(h + tx * rx);  // [L] sin(AoD)
    double* sa = sd + L;                                  // [L] sin(AoA)
    d2* g = reinterpret_cast<d2*>(sa + L);                // [L] gains (2L doubles keep 16-B alignment)
    __shared__ double red[16];
    const int c = blockIdx.x;
    const long long real = first + c;
    const int n = tx * rx;
    if (threadIdx.x == 0) {
        double nn = 0.0;
        for (int l = 0; l < L; ++l) {
            const double aod = (u01(seed, stream_id(ST_ANGLES, real), l) - 0.5) * 95.0;
            const double aoa = (u01(seed, stream_id(ST_ANGLES, real), L + l) - 0.5) * 95.0;
            sd[l] = sin(aod * M_PI / 180.0);
            sa[l] = sin(aoa * M_PI / 180.0);
            const d2 z = nrm2(seed, stream_id(ST_GAINS, real), l);
            g[l] = make_double2(z.x * M_SQRT1_2, z.y * M_SQRT1_2);
            nn += cabs2(g[l]);
        }
        nn = sqrt(nn);
        for (int l = 0; l < L; ++l) g[l] = cscale(g[l], 1.0 / nn);
    }
    __syncthreads();
    // H[r][t] = sum_l g_l exp(-j kap sinA_l r) exp(+j kap sinD_l t); vecH[r + Nr*t] (Nr = rx)
    const double kap = 2.0 * M_PI * lam_d;
    double nh = 0.0;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        const int r = k % rx, t = k / rx;
        d2 s = make_double2(0.0, 0.0);
        for (int l = 0; l < L; ++l) {
            const double ph = kap * (sd[l] * t - sa[l] * r);
            double sn, cs;
            sincos(ph, &sn, &cs);
            s = cadd(s, cmul(g[l], make_double2(cs, sn)));
        }
        h[k] = s;
        nh += cabs2(s);
        reinterpret_cast<d2*>(vecHp)[(long long)c * n + k] = s;
    }
    nh = wave_sum(nh);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = nh;
    __syncthreads();
    double nH = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) nH += red[w];
    nH = sqrt(nH);
    // X0 = vecH + x0_noise * ||vecH|| / sqrt(n) * CN(0,1)
    const double xs = x0_noise * nH / sqrt((double)n) * M_SQRT1_2;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        const d2 z = nrm2(seed, stream_id(ST_X0, real), k);
        reinterpret_cast<d2*>(X0p)[(long long)c * n + k] = cadd(h[k], cscale(z, xs));
    }
    // B = |A vecH + w|, one wave per row
    const d2* A = reinterpret_cast<const d2*>(Ap) + (a_shared ? 0LL : (long long)c * m * n);
    const double ns = sqrt(sigma2) * M_SQRT1_2;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int i = wv; i < m; i += nw) {
        d2 s = make_double2(0.0, 0.0);
        for (int k = lane; k < n; k += 64) s = cadd(s, cmul(A[(long long)i * n + k], h[k]));
        s.x = wave_sum(s.x);
        s.y = wave_sum(s.y);
        if (lane == 0) {
            const d2 z = nrm2(seed, stream_id(ST_NOISE, real), i);
            const d2 y = cadd(s, cscale(z, ns));
            Bp[(long long)c * m + i] = sqrt(cabs2(y));
        }
    }
    // InferADMM always sees B / ||B|| (inferLowRankV4_multi.m:32-38; A is already
    // at ||A||_F = sqrt(m)): normalise B, and X0 / vecH to the same scale.
    __syncthreads();
    double nb = 0.0;
    for (int i = threadIdx.x; i < m; i += blockDim.x) nb += Bp[(long long)c * m + i] * Bp[(long long)c * m + i];
    nb = wave_sum(nb);
    __syncthreads();
    if (lane == 0) red[wv] = nb;
    __syncthreads();
    nb = 0.0;
    for (int w = 0; w < nw; ++w) nb += red[w];
    const double inb = 1.0 / sqrt(nb);
    for (int i = threadIdx.x; i < m; i += blockDim.x) Bp[(long long)c * m + i] *= inb;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        d2* x0 = reinterpret_cast<d2*>(X0p) + (long long)c * n + k;
        d2* vh = reinterpret_cast<d2*>(vecHp) + (long long)c * n + k;
        *x0 = cscale(*x0, inb);
        *vh = cscale(*vh, inb);
    }
}
}  // namespace

void launch_synth_codebook(uint64_t seed, long long first, int count, int m, int n, double* A, hipStream_t st) {
    const long long total = (long long)count * m * n;
    long long blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(codebook_kernel, dim3((unsigned)blocks), dim3(256), 0, st, seed, first, count, m, n, A);
}

void launch_synth_channels(uint64_t seed, long long first, int count, int m, int tx, int rx, int L, double snr_db,
                           double x0_noise, const double* A, int a_shared, double* vecH, double* B, double* X0,
                           hipStream_t st) {
    const double sigma2 = pow(10.0, -snr_db / 10.0);
    const double lam = 3e8 / 60.48e9, d = 3.055e-3;  // A2only.m:40-41
    const size_t sh = (size_t)tx * rx * sizeof(d2) + (2 * L + 2) * sizeof(double) + L * sizeof(d2) + 16;
    hipLaunchKernelGGL(channel_kernel, dim3(count), dim3(256), sh, st, seed, first, m, tx, rx, L, sigma2, x0_noise, A,
                       a_shared, vecH, B, X0, d / lam);
}

}  // namespace ace

// Probe: f64 MFMA 16x16x4 throughput vs waves per SIMD and independent accumulators
// per wave (diagnostic only).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef double d4 __attribute__((ext_vector_type(4)));
template <int NACC, bool BUMP>
__global__ __launch_bounds__(256) void rate(double* out, int iters) {
    const int l = threadIdx.x;
    double a = 1.0 + l * 1e-3, b = 1.0 - l * 1e-3;
    d4 c[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) c[i] = d4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
        if (BUMP) a += 1e-9;
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += c[i][0];
    if (s == 12345.678) out[blockIdx.x] = s;
}
template <int NACC, bool BUMP = false>
void run(int cus, int wps, double* o, int mult) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4096 / NACC * 4 * mult;
    const int blocks = cus * wps;
    rate<NACC, BUMP><<<blocks, 256>>>(o, 16);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    rate<NACC, BUMP><<<blocks, 256>>>(o, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double fl = (double)blocks * 4 * iters * NACC * 2048.0;
    printf("bump=%d waves/SIMD=%d acc=%2d: %6.2f TF/s  cycles/MFMA/SIMD=%.1f\n", (int)BUMP, wps, NACC, fl / ms / 1e9,
           ms * 1e-3 * 2.4e9 / ((double)wps * iters * NACC));
}
int main(int argc, char** argv) {
    const int mult = argc > 1 ? atoi(argv[1]) : 1;
    int dev;
    hipGetDevice(&dev);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, dev);
    double* o;
    hipMalloc(&o, 1 << 20);
    for (int w : {2, 4, 8, 2, 4, 8}) {
        run<1>(p.multiProcessorCount, w, o, mult);
        run<4>(p.multiProcessorCount, w, o, mult);
        run<8>(p.multiProcessorCount, w, o, mult);
        run<16>(p.multiProcessorCount, w, o, mult);
    }
    run<4, true>(p.multiProcessorCount, 2, o, mult);
    run<4, true>(p.multiProcessorCount, 8, o, mult);
    return 0;
}

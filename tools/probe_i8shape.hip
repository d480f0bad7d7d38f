// Probe: v_mfma_i32_32x32x32_i8 throughput in the work-group shape of the digit-plane
// applies (512 threads, one work-group per CU, 8 accumulators per wave), with operands
// from registers, with A fragments from LDS, and with the per-block f64 epilogue.
// Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int i4v __attribute__((ext_vector_type(4)));
typedef int i16v __attribute__((ext_vector_type(16)));
#define CK(x) do { hipError_t e_ = (x); if (e_) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int MODE>   // 0: registers only; 1: A from LDS; 2: A from LDS + epilogue every 16 K-steps
__global__ __launch_bounds__(512, 1) void shape(double* out, int ksteps) {
    __shared__ __attribute__((aligned(16))) int8_t As[128 * 528];
    const int t = threadIdx.x, lane = t & 63;
    for (int i = t; i < 128 * 528 / 4; i += 512) reinterpret_cast<int*>(As)[i] = i * 2654435761u;
    __syncthreads();
    i16v acc[4][2];
#pragma unroll
    for (int R = 0; R < 4; ++R) acc[R][0] = acc[R][1] = i16v{};
    i4v b0 = {lane, 1, 2, 3}, b1 = {3, lane, 1, 7};
    i4v ar[4] = {{1, lane, 3, 4}, {lane, 2, 2, 1}, {5, 6, lane, 8}, {1, 1, 1, lane}};
    const int8_t* arow = &As[(lane & 31) * 528 + 16 * (lane >> 5)];
    double sink = 0.0;
    for (int k = 0; k < ksteps; ++k) {
        i4v af[4];
#pragma unroll
        for (int R = 0; R < 4; ++R)
            af[R] = MODE == 0 ? ar[R] : *reinterpret_cast<const i4v*>(arow + 32 * R * 528 + 32 * (k & 15));
#pragma unroll
        for (int R = 0; R < 4; ++R) {
            acc[R][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[R], b0, acc[R][0], 0, 0, 0);
            acc[R][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[R], b1, acc[R][1], 0, 0, 0);
        }
        if (MODE == 2 && (k & 15) == 15) {
#pragma unroll
            for (int R = 0; R < 4; ++R)
#pragma unroll
                for (int c = 0; c < 2; ++c)
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        double v = (double)acc[R][c][8 * q + 7];
#pragma unroll
                        for (int tt = 6; tt >= 0; --tt) v = fma(v, 128.0, (double)acc[R][c][8 * q + tt]);
                        out[((long long)blockIdx.x * 16 + 4 * R + 2 * c + q) * 512 + (t & 511)] = v;
                    }
#pragma unroll
            for (int R = 0; R < 4; ++R) acc[R][0] = acc[R][1] = i16v{};
        }
    }
#pragma unroll
    for (int R = 0; R < 4; ++R) sink += acc[R][0][0] + acc[R][1][5];
    if (sink == 1234.5) out[0] = sink;
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    double* o;
    CK(hipMalloc(&o, (size_t)cus * 4 * 16 * 512 * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int ks = 64;   // one apply_AH work-group: 4 blocks x 16 K-steps
    for (int mode = 0; mode < 3; ++mode)
        for (int mult : {1, 2}) {
            const int grid = cus * mult;
            auto go = [&]() {
                if (mode == 0) shape<0><<<grid, 512>>>(o, ks);
                else if (mode == 1) shape<1><<<grid, 512>>>(o, ks);
                else shape<2><<<grid, 512>>>(o, ks);
            };
            go();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int r = 0; r < 20; ++r) go();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double ops = 2.0 * 32768 * 8 * 8 * ks * grid;
            printf("mode %d grid %d: %.1f us/launch, %.0f TOPS\n", mode, grid, 1e3 * ms / 20, ops / (ms / 20 * 1e-3) / 1e12);
        }
    return 0;
}

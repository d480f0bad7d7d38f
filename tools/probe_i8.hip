// Probe: int8 MFMA (v_mfma_i32_32x32x32_i8, v_mfma_i32_16x16x64_i8) operand lane maps
// checked with asymmetric exact integer data under candidate k-orders, plus the issue
// rate of both shapes on gfx950.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
typedef int i4 __attribute__((ext_vector_type(4)));
typedef int i16 __attribute__((ext_vector_type(16)));
#define CK(x) do{hipError_t e=(x); if(e){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

// k index of byte j (0..15) of lane half h under hypothesis H
__device__ __host__ inline int kmap(int H, int h, int j, int kh) {   // kh = K / (number of lane groups)
    if (H == 0) return kh * h + j;                          // contiguous 16 per group
    return 8 * h + (j & 7) + (kh == 16 ? 16 : 32) * (j >> 3); // two 8-byte halves interleaved
}

template <int H>
__global__ void l32(const int8_t* A, const int8_t* B, int* D) {   // A[32][32] (row, k), B[32][32] (k, col)
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    i4 a, b;
    int8_t* pa = (int8_t*)&a;
    int8_t* pb = (int8_t*)&b;
    for (int j = 0; j < 16; ++j) {
        const int k = kmap(H, h, j, 16);
        pa[j] = A[r * 32 + k];
        pb[j] = B[k * 32 + r];
    }
    i16 c = {};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    for (int g = 0; g < 16; ++g) {
        const int row = (g & 3) + 8 * (g >> 2) + 4 * h, col = r;
        D[row * 32 + col] = c[g];
    }
}
template <int H>
__global__ void l16(const int8_t* A, const int8_t* B, int* D) {   // A[16][64], B[64][16]
    const int l = threadIdx.x, r = l & 15, h = l >> 4;
    i4 a, b;
    int8_t* pa = (int8_t*)&a;
    int8_t* pb = (int8_t*)&b;
    for (int j = 0; j < 16; ++j) {
        const int k = kmap(H, h, j, 16);
        pa[j] = A[r * 64 + k];
        pb[j] = B[k * 16 + r];
    }
    i4 c = {};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    for (int g = 0; g < 4; ++g) D[(4 * h + g) * 16 + r] = c[g];
}

__global__ void rate32(int* out, int iters) {
    const int l = threadIdx.x;
    i4 a = {l, l + 1, l + 2, l + 3}, b = {l ^ 5, l, 7, l};
    i16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c3, 0, 0, 0);
    }
    const int s = c0[0] + c1[1] + c2[2] + c3[3];
    if (s == 123456789) out[blockIdx.x] = s;
}
__global__ void rate16(int* out, int iters) {
    const int l = threadIdx.x;
    i4 a = {l, l + 1, l + 2, l + 3}, b = {l ^ 5, l, 7, l};
    i4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c3, 0, 0, 0);
    }
    const int s = c0[0] + c1[1] + c2[2] + c3[3];
    if (s == 123456789) out[blockIdx.x] = s;
}

int main() {
    int8_t hA[1024], hB[1024];
    for (int i = 0; i < 1024; ++i) {
        hA[i] = (int8_t)((i * 37 + 11) % 255 - 127);
        hB[i] = (int8_t)((i * 53 + 7) % 251 - 125);
    }
    int8_t *dA, *dB;
    int* dD;
    CK(hipMalloc(&dA, 1024));
    CK(hipMalloc(&dB, 1024));
    CK(hipMalloc(&dD, 4096 * 4));
    CK(hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice));
    int hD[1024];
    for (int H = 0; H < 2; ++H) {
        // 32x32x32
        if (H == 0) l32<0><<<1, 64>>>(dA, dB, dD); else l32<1><<<1, 64>>>(dA, dB, dD);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(hD, dD, 1024 * 4, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int i = 0; i < 32; ++i)
            for (int j = 0; j < 32; ++j) {
                int s = 0;
                for (int k = 0; k < 32; ++k) s += hA[i * 32 + k] * hB[k * 32 + j];
                bad += (s != hD[i * 32 + j]);
            }
        printf("32x32x32 i8 hypothesis %d: %d / 1024 mismatches\n", H, bad);
        // 16x16x64
        if (H == 0) l16<0><<<1, 64>>>(dA, dB, dD); else l16<1><<<1, 64>>>(dA, dB, dD);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(hD, dD, 256 * 4, hipMemcpyDeviceToHost));
        bad = 0;
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 16; ++j) {
                int s = 0;
                for (int k = 0; k < 64; ++k) s += hA[i * 64 + k] * hB[k * 16 + j];
                bad += (s != hD[i * 16 + j]);
            }
        printf("16x16x64 i8 hypothesis %d: %d / 256 mismatches\n", H, bad);
    }
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount, iters = 20000;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int s = 0; s < 2; ++s) {
        const int grid = cus * 8;   // 8 waves per CU = 2 per SIMD
        rate32<<<grid, 64>>>(dD, 10);
        rate16<<<grid, 64>>>(dD, 10);
        CK(hipDeviceSynchronize());
        float ms;
        CK(hipEventRecord(e0));
        if (s == 0) rate32<<<grid, 64>>>(dD, iters); else rate16<<<grid, 64>>>(dD, iters);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double macs = (double)grid * iters * 4 * 32768.0;
        printf("%s: %.1f TOPS (%.3f ms)\n", s == 0 ? "32x32x32 i8" : "16x16x64 i8", 2.0 * macs / (ms * 1e-3) / 1e12, ms);
    }
    return 0;
}

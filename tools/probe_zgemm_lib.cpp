// Calibration probe (diagnostic only): rocBLAS ZGEMM throughput on the unit's apply_A shape
// (C[m x batch] = A[m x n] * V[n x batch], m = 256, n = 1024, batch = 4096), complex f64.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <cstdio>
#include <vector>
int main() {
    const int m = 256, n = 1024, nb = 4096;
    rocblas_handle h;
    rocblas_create_handle(&h);
    rocblas_double_complex *A, *V, *C;
    hipMalloc(&A, sizeof(*A) * (size_t)m * n);
    hipMalloc(&V, sizeof(*V) * (size_t)n * nb);
    hipMalloc(&C, sizeof(*C) * (size_t)m * nb);
    hipMemset(A, 0, sizeof(*A) * (size_t)m * n);
    hipMemset(V, 0, sizeof(*V) * (size_t)n * nb);
    rocblas_double_complex one = {1.0, 0.0}, zero = {0.0, 0.0};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int trans = 0; trans < 2; ++trans) {
        // trans 0: C(m x nb) = A(m x n) V(n x nb)   [apply_A];  trans 1: C(n x nb) = A^H V'(m x nb) [apply_AH]
        const int M = trans ? n : m, K = trans ? m : n;
        for (int it = 0; it < 3; ++it)
            rocblas_zgemm(h, trans ? rocblas_operation_conjugate_transpose : rocblas_operation_none, rocblas_operation_none,
                          M, nb, K, &one, A, m, V, K, &zero, C, M);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        const int reps = 20;
        for (int it = 0; it < reps; ++it)
            rocblas_zgemm(h, trans ? rocblas_operation_conjugate_transpose : rocblas_operation_none, rocblas_operation_none,
                          M, nb, K, &one, A, m, V, K, &zero, C, M);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double t = ms / reps * 1e-3;
        printf("rocblas_zgemm %s M=%d N=%d K=%d: %.3f ms  %.2f TF/s (8 flops / complex MAC)\n", trans ? "A^H" : "A  ", M, nb,
               K, t * 1e3, 8.0 * M * nb * K / t / 1e12);
    }
    return 0;
}

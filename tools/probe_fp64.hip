// Probe: f64 MFMA 16x16x4 operand/accumulator lane maps (asymmetric data),
// f64 MFMA and f64 VALU FMA throughput on gfx950. Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

// A[i][k] = 1+i+100*k (16x4), B[k][j] = 1000*k + j*j (4x16); D = A*B (16x16)
__global__ void layout_k(double* out){
  int l = threadIdx.x;
  double a = 1.0 + (l&15) + 100.0*(l>>4);       // guess: A[i=l&15][k=l>>4]
  double b = 1000.0*(l>>4) + (double)((l&15)*(l&15)); // guess: B[k=l>>4][j=l&15]
  d4 acc = {0,0,0,0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0,0,0);
  for(int r=0;r<4;r++) out[l*4+r] = acc[r];
}

__global__ void mfma_rate(double* out, int iters){
  int l = threadIdx.x;
  double a = 1.0 + l*1e-3, b = 1.0 - l*1e-3;
  d4 c0={0,0,0,0},c1=c0,c2=c0,c3=c0;
  for(int i=0;i<iters;i++){
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a,b,c0,0,0,0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a,b,c1,0,0,0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a,b,c2,0,0,0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a,b,c3,0,0,0);
  }
  double s = c0[0]+c1[1]+c2[2]+c3[3];
  if (s == 12345.678) out[blockIdx.x] = s;
}

__global__ void valu_rate(double* out, int iters){
  int l = threadIdx.x + blockIdx.x*blockDim.x;
  double x0=l*1e-9,x1=x0+1,x2=x0+2,x3=x0+3,x4=x0+4,x5=x0+5,x6=x0+6,x7=x0+7;
  const double m=0.999999, a=1e-7;
  for(int i=0;i<iters;i++){
    x0=fma(x0,m,a);x1=fma(x1,m,a);x2=fma(x2,m,a);x3=fma(x3,m,a);
    x4=fma(x4,m,a);x5=fma(x5,m,a);x6=fma(x6,m,a);x7=fma(x7,m,a);
  }
  double s=x0+x1+x2+x3+x4+x5+x6+x7;
  if (s == 12345.678) out[l] = s;
}

__global__ void copy_k(const double4* __restrict__ in, double4* __restrict__ out, size_t n){
  size_t i = blockIdx.x*(size_t)blockDim.x + threadIdx.x;
  size_t st = (size_t)gridDim.x*blockDim.x;
  for(; i<n; i+=st) out[i] = in[i];
}

int main(){
  double *d; CK(hipMalloc(&d, 64*4*8));
  layout_k<<<1,64>>>(d); CK(hipDeviceSynchronize());
  double h[256]; CK(hipMemcpy(h,d,sizeof(h),hipMemcpyDeviceToHost));
  double D[16][16];
  for(int i=0;i<16;i++)for(int j=0;j<16;j++){double s=0;for(int k=0;k<4;k++) s+=(1.0+i+100.0*k)*(1000.0*k+j*j); D[i][j]=s;}
  int okA=0, okB=0;
  for(int l=0;l<64;l++)for(int r=0;r<4;r++){
    int col=l&15;
    int rowA=(l>>4)+4*r;      // guide's f64 map
    int rowB=4*(l>>4)+r;      // f32-style map
    if (fabs(h[l*4+r]-D[rowA][col])<1e-6) okA++;
    if (fabs(h[l*4+r]-D[rowB][col])<1e-6) okB++;
  }
  printf("layout: row=(l>>4)+4r matches %d/256 ; row=4(l>>4)+r matches %d/256\n", okA, okB);

  hipEvent_t e0,e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int dev; hipGetDevice(&dev); hipDeviceProp_t p; hipGetDeviceProperties(&p,dev);
  int cus = p.multiProcessorCount; printf("CUs=%d clock=%d kHz name=%s\n", cus, p.clockRate, p.gcnArchName);
  double* o; CK(hipMalloc(&o, 1<<24));
  int iters=20000; int blocks=cus*8;
  mfma_rate<<<blocks,256>>>(o, 100); CK(hipDeviceSynchronize());
  hipEventRecord(e0); mfma_rate<<<blocks,256>>>(o, iters); hipEventRecord(e1); CK(hipEventSynchronize(e1));
  float ms; hipEventElapsedTime(&ms,e0,e1);
  double fl = (double)blocks*4 /*waves*/ *iters*4*2048.0;
  printf("MFMA f64 16x16x4: %.2f TFLOP/s (%.3f ms)\n", fl/ms/1e9, ms);
  valu_rate<<<blocks,256>>>(o, 100); CK(hipDeviceSynchronize());
  hipEventRecord(e0); valu_rate<<<blocks,256>>>(o, iters); hipEventRecord(e1); CK(hipEventSynchronize(e1));
  hipEventElapsedTime(&ms,e0,e1);
  fl = (double)blocks*256*iters*8*2.0;
  printf("VALU f64 fma: %.2f TFLOP/s (%.3f ms)\n", fl/ms/1e9, ms);
  size_t n = (size_t)1<<27; // 4 GiB of double4? 2^27*32B=4GiB
  double4 *a,*b; CK(hipMalloc(&a,n*32)); CK(hipMalloc(&b,n*32)); CK(hipMemset(a,0,n*32));
  copy_k<<<cus*8,256>>>(a,b,n); CK(hipDeviceSynchronize());
  hipEventRecord(e0); for(int r=0;r<5;r++) copy_k<<<cus*8,256>>>(a,b,n); hipEventRecord(e1); CK(hipEventSynchronize(e1));
  hipEventElapsedTime(&ms,e0,e1);
  printf("copy: %.2f TB/s\n", 5.0*2*n*32/ms/1e9);
  return 0;
}

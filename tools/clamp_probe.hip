// Probe: what the VOP3 clamp bit does to v_fma_f32 / v_pk_fma_f32 results on this GPU, and the
// throughput slicer's clamp-form level computation on sample inputs.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x2 __attribute__((ext_vector_type(2)));
__global__ void k(const float* in, float* out, int n) {
    int i = threadIdx.x;
    if (i >= n) return;
    float x = in[i], r1, r3;
    asm volatile("v_fma_f32 %0, %1, %2, %3 clamp" : "=v"(r1) : "v"(x), "v"(1.0f), "v"(0.0f));
    f32x2 xv = f32x2{x, -x}, r2;
    f32x2 one = f32x2{1.f, 1.f}, zero = f32x2{0.f, 0.f};
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3 clamp" : "=v"(r2) : "v"(xv), "v"(one), "v"(zero));
    asm volatile("v_add_f32_e64 %0, %1, 0 clamp" : "=v"(r3) : "v"(x));
    out[5 * i + 0] = r1;
    out[5 * i + 1] = r2.x;
    out[5 * i + 2] = r2.y;
    out[5 * i + 3] = r3;
    out[5 * i + 4] = __builtin_amdgcn_fmed3f(x, 0.f, 1.f);
}
int main() {
    const int n = 8;
    float h[n] = {-2.f, -0.25f, 0.f, 0.3f, 0.99f, 1.f, 1.5f, 7.f}, o[5 * n];
    float *din, *dout;
    hipMalloc(&din, sizeof h);
    hipMalloc(&dout, sizeof o);
    hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout, n);
    hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    printf("x fma_clamp pk_clamp(x) pk_clamp(-x) add_clamp med3\n");
    for (int i = 0; i < n; ++i)
        printf("%g %g %g %g %g %g\n", h[i], o[5 * i], o[5 * i + 1], o[5 * i + 2], o[5 * i + 3], o[5 * i + 4]);
    return 0;
}

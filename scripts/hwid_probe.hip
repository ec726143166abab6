#include <hip/hip_runtime.h>
__global__ void k(unsigned *o) {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    if (threadIdx.x == 0) { o[blockIdx.x * 2] = v; o[blockIdx.x * 2 + 1] = x; }
}
int main() {
    unsigned *d; hipMalloc(&d, 4096 * 8);
    hipLaunchKernelGGL(k, dim3(2048), dim3(256), 64 * 1024, 0, d);
    unsigned h[4096]; hipMemcpy(h, d, 2048 * 8, hipMemcpyDeviceToHost);
    for (int b = 0; b < 2048; b += 1) {
        unsigned v = h[2*b];
        if (b < 24 || (b >= 256 && b < 272) || (b>=504 && b < 520))
        printf("b=%d wave=%u simd=%u cu=%u sh=%u se=%u tg=%u xcc=%u\n", b, v & 15, (v >> 4) & 3, (v >> 8) & 15, (v >> 12) & 1, (v >> 13) & 7, (v >> 16) & 15, h[2*b+1] & 15);
    }
    return 0;
}

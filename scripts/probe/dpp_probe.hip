// Probe of gfx950 DPP controls (wave_shr:1, row_bcast:15/31, row_newbcast:15): prints each
// lane's result for source = lane id; bound_ctrl 0 and old = -1 marks lanes not written.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL, int ROWMASK>
__global__ void k(int* out) {
    const int l = threadIdx.x;
    out[l] = __builtin_amdgcn_update_dpp(-1, l, CTRL, ROWMASK, 0xf, false);
}
template <int CTRL, int ROWMASK>
void run(const char* name) {
    int* d; hipMalloc(&d, 64 * 4);
    hipLaunchKernelGGL((k<CTRL, ROWMASK>), dim3(1), dim3(64), 0, 0, d);
    int h[64]; hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
    printf("%-16s", name);
    for (int i = 0; i < 64; ++i) printf("%d ", h[i]);
    printf("\n");
    hipFree(d);
}
int main() {
    run<0x138, 0xf>("wave_shr1");
    run<0x13c, 0xf>("wave_ror1");
    run<0x142, 0xa>("row_bcast15");
    run<0x143, 0xc>("row_bcast31");
    run<0x15f, 0xf>("row_newbcast15");
    run<0x111, 0xf>("row_shr1");
    return 0;
}

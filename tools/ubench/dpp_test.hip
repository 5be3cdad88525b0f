#include <hip/hip_runtime.h>
__global__ void k(int* o, const int* in) {
    int x = in[threadIdx.x];
    int up = __builtin_amdgcn_update_dpp(0, x, 0x138, 0xf, 0xf, false);   // wave_shr:1
    int dn = __builtin_amdgcn_update_dpp(0, x, 0x130, 0xf, 0xf, false);   // wave_shl:1
    int v = x;
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
    o[threadIdx.x] = up; o[64 + threadIdx.x] = dn; o[128 + threadIdx.x] = v;
}
int main() {
    int *d, *di; int h[192], hi[64];
    for (int i = 0; i < 64; ++i) hi[i] = i + 1;
    hipMalloc(&d, 192 * 4); hipMalloc(&di, 64 * 4);
    hipMemcpy(di, hi, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, di);
    hipMemcpy(h, d, 192 * 4, hipMemcpyDeviceToHost);
    int ok = 1, s = 0;
    for (int i = 0; i < 64; ++i) {
        s += hi[i];
        if (h[i] != (i ? hi[i - 1] : 0)) ok = 0;
        if (h[64 + i] != (i < 63 ? hi[i + 1] : 0)) ok = 0;
        if (h[128 + i] != s) { ok = 0; printf("scan lane %d got %d want %d\n", i, h[128 + i], s); }
    }
    printf(ok ? "DPP_OK\n" : "DPP_BAD\n");
    return 0;
}

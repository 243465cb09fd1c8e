// Prints what v_permlane32_swap / v_permlane16_swap / DPP row_shl return per lane on gfx950
// (which builtin result element carries which source lane), for the descriptor's reduction trees.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* o)
{
    const int l = threadIdx.x;
    auto a = __builtin_amdgcn_permlane32_swap(l, 100 + l, false, false);
    auto b = __builtin_amdgcn_permlane16_swap(l, 100 + l, false, false);
    o[l] = a[0]; o[64 + l] = a[1]; o[128 + l] = b[0]; o[192 + l] = b[1];
    o[256 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x108, 0xF, 0xF, true);    // row_shl:8
    o[320 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x111, 0xF, 0xF, true);    // row_shr:1
    o[384 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x142, 0xF, 0xF, false);   // row_bcast:15
    o[448 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x143, 0xF, 0xF, false);   // row_bcast:31
}
int main()
{
    int* d; hipMalloc(&d, 512 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    int h[512]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* nm[8] = {"p32[0]", "p32[1]", "p16[0]", "p16[1]", "row_shl8", "row_shr1", "bcast15", "bcast31"};
    for (int r = 0; r < 8; ++r) { printf("%-9s", nm[r]); for (int l = 0; l < 64; ++l) printf(" %d", h[r * 64 + l]); printf("\n"); }
    return 0;
}

// glds_exec_probe.hip -- does an LDS-DMA (global_load_lds_dwordx4) issued
// with some lanes masked off leave those lanes' LDS bytes alone?  (The v4
// row-record kernel's spill reload depends on the answer; csrc/rows.hip.)
// One wave: LDS filled with 0xEE, a DMA of 64 x 16 bytes from a buffer of
// 0x11 with only the even lanes active, then every lane's 16 bytes printed
// as "lane: first byte".  Build: hipcc --offload-arch=gfx950 -O2 -o
// tools/_build/glds_exec_probe tools/glds_exec_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void k_probe(const uint8_t *src, uint8_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[1024];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < 1024; i += 64) lds[i] = 0xEE;
    __syncthreads();
    if ((lane & 1) == 0)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + 16 * lane),
                                         (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    for (uint32_t i = lane; i < 1024; i += 64) out[i] = lds[i];
}

int main() {
    uint8_t *src = nullptr, *out = nullptr;
    if (hipMalloc(&src, 1024) != hipSuccess || hipMalloc(&out, 1024) != hipSuccess) return 1;
    (void)hipMemset(src, 0x11, 1024);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, src, out);
    uint8_t h[1024];
    if (hipMemcpy(h, out, 1024, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int kept = 0, zeroed = 0, written = 0;
    for (int l = 1; l < 64; l += 2) {
        const uint8_t b = h[16 * l];
        kept += b == 0xEE;
        zeroed += b == 0x00;
        written += b == 0x11;
    }
    int even_ok = 0;
    for (int l = 0; l < 64; l += 2) even_ok += h[16 * l] == 0x11;
    std::printf("{\"masked_lanes\": 32, \"kept\": %d, \"zeroed\": %d, \"written\": %d, \"active_lanes_written\": %d}\n",
                kept, zeroed, written, even_ok);
    return 0;
}

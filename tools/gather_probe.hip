// gather_probe.hip -- measures the random-line read ceiling of the GPU for
// the access pattern of the BRWT traversal: independent random reads of
// `bytes` contiguous bytes (16/64/128) at line-aligned addresses of a buffer
// of `gib` GiB.  Reports lines/s and bytes/s (DESIGN.md "Measurement").
// Not part of the product; a calibration tool for the roofline.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <string>

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <int VEC, int U>
__global__ __launch_bounds__(256) void k_probe(const uint4 *__restrict__ buf, uint64_t nlines, uint32_t stride16,
                                                uint32_t iters, uint64_t seed, uint4 *out) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (uint32_t it = 0; it < iters; ++it) {
        uint4 v[U][VEC];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t line = mix64(seed ^ (tid * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)(it * U + u) << 40)) % nlines;
            const uint4 *p = buf + line * stride16;
#pragma unroll
            for (int k = 0; k < VEC; ++k) v[u][k] = p[k];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                acc.x ^= v[u][k].x; acc.y ^= v[u][k].y; acc.z ^= v[u][k].z; acc.w ^= v[u][k].w;
            }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[tid] = acc;
}

// groups of G lanes read one 16*G-byte segment of a random line together
// (the coalesced shape of the group traversal kernel)
template <int U>
__global__ __launch_bounds__(256) void k_probe_group(const uint4 *__restrict__ buf, uint64_t nlines, uint32_t G,
                                                      uint32_t iters, uint64_t seed, uint4 *out) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t grp = tid / G;
    const uint32_t c = tid % G;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (uint32_t it = 0; it < iters; ++it) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t line = mix64(seed ^ (grp * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)(it * U + u) << 40)) % nlines;
            v[u] = buf[line * 8 + c];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc.x ^= v[u].x; acc.y ^= v[u].y; acc.z ^= v[u].z; acc.w ^= v[u].w;
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[tid] = acc;
}

template <int U>
double run_group(const uint4 *buf, uint64_t bytes_total, uint32_t G, int grid, uint32_t iters, uint4 *out) {
    const uint64_t nlines = bytes_total / 128;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k_probe_group<U>, dim3(grid), dim3(256), 0, 0, buf, nlines, G, iters, 1, out);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_probe_group<U>, dim3(grid), dim3(256), 0, 0, buf, nlines, G, iters, 7, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return (double)grid * 256 / G * iters * U / (ms / 1e3);
}

template <int VEC>
double run(const uint4 *buf, uint64_t bytes_total, uint32_t line_bytes, int grid, uint32_t iters, uint4 *out) {
    const uint64_t nlines = bytes_total / line_bytes;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_probe<VEC, 4>), dim3(grid), dim3(256), 0, 0, buf, nlines, line_bytes / 16, iters, 1, out);
    hipEventRecord(a);
    hipLaunchKernelGGL((k_probe<VEC, 4>), dim3(grid), dim3(256), 0, 0, buf, nlines, line_bytes / 16, iters, 7, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double reads = (double)grid * 256 * iters * 4;
    return reads / (ms / 1e3);
}

int main(int argc, char **argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 64.0;
    const uint64_t total = (uint64_t)(gib * (1ull << 30));
    void *buf = nullptr;
    if (hipMalloc(&buf, total) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(buf, 1, total);
    uint4 *out = nullptr;
    hipMalloc(&out, (size_t)65536 * 256 * sizeof(uint4));
    hipDeviceSynchronize();
    if (argc > 2 && std::string(argv[2]) == "calib") {
        // counter calibration: ONE dispatch of k_probe_group<4> with G = 4, i.e.
        // a known number of random 64-B segment reads (the traversal's pattern);
        // FETCH_SIZE / TCC_EA0_RDREQ of that dispatch divided by the segment
        // count gives the bytes each counter tallies per 64-B random read.
        const int grid = 8192;
        const uint32_t G = 4, iters = 64;
        const uint64_t nlines = total / 128;
        hipLaunchKernelGGL(k_probe_group<4>, dim3(grid), dim3(256), 0, 0, (const uint4 *)buf, nlines, G, iters,
                           (uint64_t)11, out);
        hipDeviceSynchronize();
        printf("calib: buffer %.1f GiB, one k_probe_group<4> dispatch, G=%u: %llu random 64-B segments (%llu bytes)\n",
               gib, G, (unsigned long long)grid * 256 / G * iters * 4,
               (unsigned long long)grid * 256 / G * iters * 4 * 64);
        hipFree(buf);
        return 0;
    }
    for (int grid : {2048, 8192}) {
        const uint32_t iters = 64;
        double r16 = run<1>((const uint4 *)buf, total, 128, grid, iters, out);
        double r64 = run<4>((const uint4 *)buf, total, 128, grid, iters, out);
        double r128 = run<8>((const uint4 *)buf, total, 128, grid, iters, out);
        double r64a = run<4>((const uint4 *)buf, total, 64, grid, iters, out);
        printf("buffer %.1f GiB grid %d: 16B-in-128B-line %.2f G/s | 64B(128-aligned) %.2f G/s | 128B %.2f G/s (%.2f TB/s) | 64B(64-aligned) %.2f G/s (%.2f TB/s)\n",
               gib, grid, r16 / 1e9, r64 / 1e9, r128 / 1e9, r128 * 128 / 1e12, r64a / 1e9, r64a * 64 / 1e12);
    }
    for (uint32_t G : {1u, 2u, 4u, 8u}) {
        const int grid = 8192;
        double u1 = run_group<1>((const uint4 *)buf, total, G, grid, 64, out);
        double u4 = run_group<4>((const uint4 *)buf, total, G, grid, 64, out);
        printf("buffer %.1f GiB group G=%u (%u B segment): 1 in flight %.2f G lines/s | 4 in flight %.2f G lines/s\n",
               gib, G, 16 * G, u1 / 1e9, u4 / 1e9);
    }
    hipFree(buf);
    return 0;
}

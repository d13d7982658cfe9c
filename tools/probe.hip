// probe.hip -- measurement kernels for bench.py's roofline (not part of the
// product library): the two ceilings the traversal is compared against.
//
//   probe_stream_read  : a streaming read of a device buffer (16 B per lane,
//                        grid-stride, every byte once per pass) -> GB/s; the
//                        achievable HBM read rate beside the 8 TB/s spec.
//   probe_random64     : random 64-byte segments at 128-byte-aligned offsets of
//                        a device buffer, each segment read by 4 lanes as ONE
//                        coalesced request (the access shape of the traversal's
//                        block reads) -> requests/s; the request
//                        ceiling this access shape can reach.
// Both time themselves with HIP events on the stream they run on.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_stream_read(const u32x4 *__restrict__ buf, uint64_t n16, u32x4 *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    u32x4 acc = u32x4{0, 0, 0, 0};
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {  // 4 independent loads in flight per lane
        const u32x4 a = __builtin_nontemporal_load(buf + i);
        const u32x4 b = __builtin_nontemporal_load(buf + i + stride);
        const u32x4 c = __builtin_nontemporal_load(buf + i + 2 * stride);
        const u32x4 d = __builtin_nontemporal_load(buf + i + 3 * stride);
        acc.x ^= a.x ^ b.x ^ c.x ^ d.x;
        acc.y ^= a.y ^ b.y ^ c.y ^ d.y;
        acc.z ^= a.z ^ b.z ^ c.z ^ d.z;
        acc.w ^= a.w ^ b.w ^ c.w ^ d.w;
    }
    for (; i < n16; i += stride) {
        const u32x4 a = buf[i];
        acc.x ^= a.x;
        acc.y ^= a.y;
        acc.z ^= a.z;
        acc.w ^= a.w;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) out[0] = acc;  // keeps the loads alive
}

// groups of 4 lanes read one 64-byte segment of a random 128-byte line
// together, U segments in flight per group
template <int U>
__global__ __launch_bounds__(256) void k_random64(const u32x4 *__restrict__ buf, uint64_t nlines, uint32_t iters,
                                                  uint64_t seed, u32x4 *out) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t grp = tid / 4;
    const uint32_t c = tid % 4;
    u32x4 acc = u32x4{0, 0, 0, 0};
    for (uint32_t it = 0; it < iters; ++it) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t line = mix64(seed ^ (grp * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)(it * U + u) << 40)) % nlines;
            v[u] = __builtin_nontemporal_load(buf + line * 8 + c);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc.x ^= v[u].x;
            acc.y ^= v[u].y;
            acc.z ^= v[u].z;
            acc.w ^= v[u].w;
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) out[tid & 1023] = acc;
}


// groups of L lanes read one (16 L)-byte segment at a random (16 L)-aligned
// offset together, U segments in flight per group (the sweep behind
// bench.py's request ceiling: segment size x requests in flight x occupancy)
template <int L, int U>
__global__ __launch_bounds__(256) void k_randseg(const u32x4 *__restrict__ buf, uint64_t nseg, uint32_t iters,
                                                 uint64_t seed, u32x4 *out) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t grp = tid / L;
    const uint32_t c = tid % L;
    u32x4 acc = u32x4{0, 0, 0, 0};
    for (uint32_t it = 0; it < iters; ++it) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t s = mix64(seed ^ (grp * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)(it * U + u) << 40)) % nseg;
            v[u] = __builtin_nontemporal_load(buf + s * L + c);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc.x ^= v[u].x;
            acc.y ^= v[u].y;
            acc.z ^= v[u].z;
            acc.w ^= v[u].w;
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) out[tid & 1023] = acc;
}

// one lane per segment: each lane reads its own 64-byte segment as 4 x 16 B
// (the uncoalesced form of the same request), U segments in flight per lane
template <int U>
__global__ __launch_bounds__(256) void k_randseg_lane(const u32x4 *__restrict__ buf, uint64_t nseg, uint32_t iters,
                                                      uint64_t seed, u32x4 *out) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    u32x4 acc = u32x4{0, 0, 0, 0};
    for (uint32_t it = 0; it < iters; ++it) {
        u32x4 v[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t s = mix64(seed ^ (tid * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)(it * U + u) << 40)) % nseg;
#pragma unroll
            for (int q = 0; q < 4; ++q) v[u][q] = __builtin_nontemporal_load(buf + s * 4 + q);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                acc.x ^= v[u][q].x;
                acc.y ^= v[u][q].y;
                acc.z ^= v[u][q].z;
                acc.w ^= v[u][q].w;
            }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) out[tid & 1023] = acc;
}

}  // namespace

extern "C" {

// Streaming read of [buf, buf + bytes) `passes` times (after one untimed pass).
// Returns 0 and the rate in GB/s, or a hipError_t value.
int probe_stream_read(const void *buf, uint64_t bytes, int passes, void *stream, double *gbs) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const uint64_t n16 = bytes / 16;
    if (!buf || !n16 || passes <= 0 || !gbs) return (int)hipErrorInvalidValue;
    u32x4 *out = nullptr;
    hipError_t e = hipMalloc(&out, 1024 * sizeof(u32x4));
    if (e != hipSuccess) return (int)e;
    int cus = 0, dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int grid = (cus > 0 ? cus : 256) * 16;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k_stream_read, dim3(grid), dim3(256), 0, s, (const u32x4 *)buf, n16, out);
    (void)hipEventRecord(a, s);
    for (int p = 0; p < passes; ++p)
        hipLaunchKernelGGL(k_stream_read, dim3(grid), dim3(256), 0, s, (const u32x4 *)buf, n16, out);
    (void)hipEventRecord(b, s);
    e = hipEventSynchronize(b);
    float ms = 0;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipFree(out);
    if (e != hipSuccess) return (int)e;
    *gbs = (double)n16 * 16 * passes / (ms / 1e3) / 1e9;
    return 0;
}

// Random 64-byte segment reads over [buf, buf + bytes) (a buffer much larger
// than the 256 MiB Infinity Cache).  Returns 0 and the segments per second.
int probe_random64(const void *buf, uint64_t bytes, void *stream, double *segments_per_s) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const uint64_t nlines = bytes / 128;
    if (!buf || nlines < 2 || !segments_per_s) return (int)hipErrorInvalidValue;
    u32x4 *out = nullptr;
    hipError_t e = hipMalloc(&out, 1024 * sizeof(u32x4));
    if (e != hipSuccess) return (int)e;
    const int grid = 8192;
    const uint32_t iters = 64;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k_random64<4>, dim3(grid), dim3(256), 0, s, (const u32x4 *)buf, nlines, iters, 1ull, out);
    (void)hipEventRecord(a, s);
    hipLaunchKernelGGL(k_random64<4>, dim3(grid), dim3(256), 0, s, (const u32x4 *)buf, nlines, iters, 7ull, out);
    (void)hipEventRecord(b, s);
    e = hipEventSynchronize(b);
    float ms = 0;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipFree(out);
    if (e != hipSuccess) return (int)e;
    *segments_per_s = (double)grid * 256 / 4 * iters * 4 / (ms / 1e3);
    return 0;
}

// Random segment reads (see k_randseg): seg_bytes in {32, 64, 128, 256} (or
// 0 = 64-byte segments read lane-wise, k_randseg_lane), `inflight` in
// {1, 2, 4, 8, 16} segments per group, `grid` workgroups of `threads` lanes.
// Returns 0 and the segments per second.
int probe_random_seg(const void *buf, uint64_t bytes, int seg_bytes, int inflight, int grid, int threads,
                     void *stream, double *segments_per_s) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int L = seg_bytes ? seg_bytes / 16 : 4;
    const uint64_t nseg = bytes / (16ull * L);
    if (!buf || nseg < 2 || !segments_per_s || grid <= 0 || threads <= 0 || threads > 256 || threads % 64) return (int)hipErrorInvalidValue;
    typedef void (*Fn)(const u32x4 *, uint64_t, uint32_t, uint64_t, u32x4 *);
    Fn fn = nullptr;
#define RS(LL, UU) if (seg_bytes == 16 * LL && inflight == UU) fn = k_randseg<LL, UU>;
#define RSU(LL) RS(LL, 1) RS(LL, 2) RS(LL, 4) RS(LL, 8) RS(LL, 16)
    RSU(2) RSU(4) RSU(8) RSU(16)
#undef RSU
#undef RS
    if (seg_bytes == 0) {
        if (inflight == 1) fn = k_randseg_lane<1>;
        if (inflight == 2) fn = k_randseg_lane<2>;
        if (inflight == 4) fn = k_randseg_lane<4>;
    }
    if (!fn) return (int)hipErrorInvalidValue;
    u32x4 *out = nullptr;
    hipError_t e = hipMalloc(&out, 1024 * sizeof(u32x4));
    if (e != hipSuccess) return (int)e;
    const uint32_t lanes_per_seg = seg_bytes ? (uint32_t)L : 1u;
    // ~64 M segments per timed launch
    const uint64_t per_iter = (uint64_t)grid * threads / lanes_per_seg * inflight;
    const uint32_t iters = (uint32_t)std::max<uint64_t>(1, (64ull << 20) / per_iter);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(threads), 0, s, (const u32x4 *)buf, nseg, iters, 1ull, out);
    (void)hipEventRecord(a, s);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(threads), 0, s, (const u32x4 *)buf, nseg, iters, 7ull, out);
    (void)hipEventRecord(b, s);
    e = hipEventSynchronize(b);
    float ms = 0;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipFree(out);
    if (e != hipSuccess) return (int)e;
    *segments_per_s = (double)per_iter * iters / (ms / 1e3);
    return 0;
}

}  // extern "C"

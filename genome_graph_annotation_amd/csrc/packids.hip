// packids.hip -- bit-packing of column ids / label counts for the multi-GPU
// exchange (genome_graph_annotation_amd/dist.py): n values < 2^bits become
// ceil(n * bits / 32) u32 words, value i at bits [i*bits, (i+1)*bits),
// LSB-first.  One pass each way; the unpacking writes the int32 CSR directly.
#include <algorithm>

#include "device_access.hpp"
#include "mbrwt_internal.hpp"

namespace mbrwt {
namespace {

__global__ __launch_bounds__(256) void k_pack_ids(const uint32_t *__restrict__ in, uint64_t n, uint32_t bits,
                                                  uint32_t *__restrict__ words, uint64_t nwords) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t mask = bits == 32 ? 0xFFFFFFFFu : (1u << bits) - 1u;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nwords; k += gstride) {
        const uint64_t b0 = 32 * k, b1 = b0 + 32;  // the word's bit range
        uint64_t i = b0 / bits;
        uint32_t w = 0;
        for (; i < n && i * bits < b1; ++i) {
            const uint64_t pos = i * bits;  // value i's first bit
            const uint32_t v = gld(in + i) & mask;
            if (pos >= b0) w |= v << (pos - b0);
            else w |= v >> (b0 - pos);
        }
        gst(words + k, w);
    }
}

__global__ __launch_bounds__(256) void k_unpack_ids(const uint32_t *__restrict__ words, uint64_t n, uint32_t bits,
                                                    uint32_t *__restrict__ out) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t mask = bits == 32 ? 0xFFFFFFFFu : (1u << bits) - 1u;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        const uint64_t pos = i * bits;
        const uint64_t w = pos >> 5;
        const uint32_t off = (uint32_t)(pos & 31);
        uint32_t x = gld(words + w) >> off;
        if (off + bits > 32) x |= gld(words + w + 1) << (32 - off);
        gst(out + i, x & mask);
    }
}

// every rank's segment of an all-gathered wire buffer in one pass: segment r
// (words at base + r * stride) holds first[r+1] - first[r] values, which go
// to out[first[r] ..)
constexpr uint32_t kMaxSegs = 64;
struct Segs {
    uint64_t first[kMaxSegs + 1];
};
__global__ __launch_bounds__(256) void k_unpack_segments(const uint8_t *__restrict__ base, uint64_t stride,
                                                         uint32_t nseg, Segs sg, uint32_t bits,
                                                         uint32_t *__restrict__ out) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t mask = bits == 32 ? 0xFFFFFFFFu : (1u << bits) - 1u;
    const uint64_t N = sg.first[nseg];
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gstride) {
        uint32_t lo = 0, hi = nseg;  // the last r with first[r] <= i
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (sg.first[mid] <= i) lo = mid;
            else hi = mid;
        }
        const uint32_t *words = reinterpret_cast<const uint32_t *>(base + lo * stride);
        const uint64_t pos = (i - sg.first[lo]) * bits;
        const uint64_t w = pos >> 5;
        const uint32_t off = (uint32_t)(pos & 31);
        uint32_t x = gld(words + w) >> off;
        if (off + bits > 32) x |= gld(words + w + 1) << (32 - off);
        gst(out + i, x & mask);
    }
}

unsigned grid_of(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 16384)); }

}  // namespace
}  // namespace mbrwt

using namespace mbrwt;

extern "C" {

int mbrwt_pack_ids_device(const uint32_t *d_values, uint64_t n, uint32_t bits, uint32_t *d_words, void *stream) {
    if (bits < 1 || bits > 32 || (n && (!d_values || !d_words))) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    const uint64_t nwords = (n * bits + 31) / 32;
    if (nwords) {
        hipLaunchKernelGGL(k_pack_ids, dim3(grid_of(nwords)), dim3(256), 0, (hipStream_t)stream, d_values, n, bits,
                           d_words, nwords);
        MBRWT_HIP(hipGetLastError());
    }
    return MBRWT_OK;
}

int mbrwt_unpack_ids_device(const uint32_t *d_words, uint64_t n, uint32_t bits, uint32_t *d_values, void *stream) {
    if (bits < 1 || bits > 32 || (n && (!d_values || !d_words))) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    if (n) {
        hipLaunchKernelGGL(k_unpack_ids, dim3(grid_of(n)), dim3(256), 0, (hipStream_t)stream, d_words, n, bits,
                           d_values);
        MBRWT_HIP(hipGetLastError());
    }
    return MBRWT_OK;
}

int mbrwt_unpack_segments_device(const void *d_base, uint32_t nseg, uint64_t seg_stride, const uint64_t *counts,
                                 uint32_t bits, uint32_t *d_values, void *stream) {
    if (bits < 1 || bits > 32 || (nseg && (!d_base || !counts)) || (seg_stride % 4)) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    uint64_t done = 0;
    for (uint32_t r0 = 0; r0 < nseg; r0 += kMaxSegs) {  // (more than 64 ranks: one launch per 64)
        const uint32_t k = std::min<uint32_t>(kMaxSegs, nseg - r0);
        Segs sg{};
        for (uint32_t r = 0; r < k; ++r) sg.first[r + 1] = sg.first[r] + counts[r0 + r];
        if (sg.first[k] && !d_values) {
            set_error("invalid argument");
            return MBRWT_ERR_INVALID;
        }
        if (sg.first[k]) {
            hipLaunchKernelGGL(k_unpack_segments, dim3(grid_of(sg.first[k])), dim3(256), 0, (hipStream_t)stream,
                               reinterpret_cast<const uint8_t *>(d_base) + r0 * seg_stride, seg_stride, k, sg, bits,
                               d_values + done);
            MBRWT_HIP(hipGetLastError());
        }
        done += sg.first[k];
    }
    return MBRWT_OK;
}

}  // extern "C"

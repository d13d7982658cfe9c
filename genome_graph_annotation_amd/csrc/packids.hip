// packids.hip -- bit-packing of column ids / label counts for the multi-GPU
// exchange (genome_graph_annotation_amd/dist.py): n values < 2^bits become
// ceil(n * bits / 32) u32 words, value i at bits [i*bits, (i+1)*bits),
// LSB-first.  One pass each way; the unpacking writes the int32 CSR directly.
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

}  // extern "C"

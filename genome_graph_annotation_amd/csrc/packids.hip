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

// a rank's wire segment with its label count on the device (include/mbrwt.h
// mbrwt_pack_csr_device): header, row counts from the offsets, labels; one
// grid-stride pass over the count words and the label words, one output word
// per thread (measured faster than 32-value chunks per thread with 16-byte
// loads: 0.19 vs 0.24 ms for 8 M rows -- lanes 128 bytes apart coalesce badly)
__global__ __launch_bounds__(256) void k_pack_csr(const uint64_t *__restrict__ offsets, uint64_t n_rows,
                                                  const uint32_t *__restrict__ cols, uint64_t cols_cap,
                                                  const uint64_t *__restrict__ num_labels, uint64_t cap,
                                                  uint32_t bits_c, uint32_t bits_l, uint32_t *__restrict__ wire,
                                                  uint64_t lab_word0, uint64_t cnt_words, uint64_t lab_words) {
    const uint64_t L = gld(num_labels);
    // more labels than the rank's own CSR holds: its get_rows failed with
    // MBRWT_ERR_CAPACITY and left the CSR unwritten -- the header carries a
    // count over every capacity (the unpack flags the exchange) and nothing
    // is read from the CSR
    const bool lost = L > cols_cap;
    const uint64_t nl = lost ? 0 : L < cap ? L : cap;
    const uint64_t hdr = lost ? ~0ull : L;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        gst(wire, (uint32_t)hdr);
        gst(wire + 1, (uint32_t)(hdr >> 32));
    }
    if (lost) return;
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t total = cnt_words + lab_words;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total; k += gstride) {
        const bool lab = k >= cnt_words;
        const uint64_t kk = lab ? k - cnt_words : k;
        const uint32_t bits = lab ? bits_l : bits_c;
        const uint64_t n = lab ? nl : n_rows;
        const uint32_t mask = bits == 32 ? 0xFFFFFFFFu : (1u << bits) - 1u;
        const uint64_t b0 = 32 * kk, b1 = b0 + 32;
        uint32_t w = 0;
        for (uint64_t i = b0 / bits; i < n && i * bits < b1; ++i) {
            const uint64_t pos = i * bits;
            const uint32_t v = (lab ? gld(cols + i) : (uint32_t)(gld(offsets + i + 1) - gld(offsets + i))) & mask;
            if (pos >= b0) w |= v << (pos - b0);
            else w |= v >> (b0 - pos);
        }
        gst(wire + (lab ? lab_word0 + kk : 2 + kk), w);
    }
}

// the labels of every segment, the segments' sizes from their headers.
// A workgroup writes global labels [2048 g, 2048 g + 2048): when they lie in
// one segment (nearly always), their packed bits are staged in LDS by
// coalesced word loads and every thread extracts labels t, t + 256, ...
// (coalesced stores); else label by label.
constexpr uint32_t kUnpackTile = 2048;
__global__ __launch_bounds__(256) void k_unpack_labels_dev(const uint8_t *__restrict__ base, uint64_t stride,
                                                           uint32_t nseg, uint64_t lab_off, uint64_t cap,
                                                           uint32_t bits, uint32_t *__restrict__ out,
                                                           uint64_t out_cap, unsigned long long *status) {
    __shared__ uint64_t first[kMaxSegs + 1];
    __shared__ uint32_t bad;
    __shared__ uint32_t stage[kUnpackTile + 2];  // (bits <= 32: at most 2048 + 1 words)
    if (threadIdx.x < 64) {  // the headers, one lane each, then a wave scan
        const uint32_t r = threadIdx.x;
        uint64_t L = 0;
        if (r < nseg) {
            const uint32_t *h = reinterpret_cast<const uint32_t *>(base + r * stride);
            L = (uint64_t)gld(h) | ((uint64_t)gld(h + 1) << 32);
        }
        const bool over = L > cap;
        const uint64_t Lc = L < cap ? L : cap;
        uint64_t x = Lc;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(x, d, 64);
            if (r >= d) x += y;
        }
        if (r < nseg) first[r + 1] = x;
        if (r == 0) first[0] = 0;
        const uint64_t tot = __shfl(x, 63, 64);
        const bool any_over = __any(over);
        if (r == 0) {
            bad = (any_over || tot > out_cap) ? 1u : 0u;
            if (blockIdx.x == 0) {
                status[0] = tot;
                status[1] = bad;
            }
        }
    }
    __syncthreads();
    if (bad) return;
    const uint64_t N = first[nseg];
    const uint32_t mask = bits == 32 ? 0xFFFFFFFFu : (1u << bits) - 1u;
    for (uint64_t g = blockIdx.x; (uint64_t)kUnpackTile * g < N; g += gridDim.x) {
        const uint64_t i0 = (uint64_t)kUnpackTile * g;
        const uint64_t i1 = i0 + kUnpackTile < N ? i0 + kUnpackTile : N;
        uint32_t lo = 0, hi = nseg;  // the segment of label i0
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (first[mid] <= i0) lo = mid;
            else hi = mid;
        }
        const uint32_t *words = reinterpret_cast<const uint32_t *>(base + lo * stride + lab_off);
        if (i1 <= first[lo + 1]) {
            const uint64_t b0 = (i0 - first[lo]) * bits;
            const uint64_t w0 = b0 >> 5;
            const uint32_t sh = (uint32_t)(b0 & 31);
            const uint32_t nw = (uint32_t)(((i1 - i0) * bits + sh + 31) >> 5);
            for (uint32_t k = threadIdx.x; k < nw; k += 256) stage[k] = gld(words + w0 + k);
            __syncthreads();
            for (uint32_t j = threadIdx.x; j < (uint32_t)(i1 - i0); j += 256) {
                const uint32_t pos = sh + j * bits, w = pos >> 5, off = pos & 31;
                uint32_t x = stage[w] >> off;
                if (off + bits > 32) x |= stage[w + 1] << (32 - off);
                gst(out + i0 + j, x & mask);
            }
            __syncthreads();  // the stage is refilled for the next tile
        } else {
            for (uint64_t i = i0 + threadIdx.x; i < i1; i += 256) {
                uint32_t s2 = lo;
                while (s2 + 1 < nseg && first[s2 + 1] <= i) ++s2;
                const uint32_t *wd = reinterpret_cast<const uint32_t *>(base + s2 * stride + lab_off);
                const uint64_t pos = (i - first[s2]) * bits;
                const uint64_t w = pos >> 5;
                const uint32_t off = (uint32_t)(pos & 31);
                uint32_t x = gld(wd + w) >> off;
                if (off + bits > 32) x |= gld(wd + w + 1) << (32 - off);
                gst(out + i, x & mask);
            }
        }
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

uint64_t mbrwt_wire_labels_offset(uint64_t n_rows, uint32_t bits_count) {
    if (bits_count < 1 || bits_count > 32) return 0;
    return (8 + (n_rows + 31) / 32 * bits_count * 4 + 15) / 16 * 16;  // (whole 32-value chunks)
}

int mbrwt_pack_csr_device(const uint64_t *d_offsets, uint64_t n_rows, const uint32_t *d_cols, uint64_t cols_cap,
                          const uint64_t *d_num_labels, uint64_t labels_cap, uint32_t bits_count, uint32_t bits_label,
                          uint64_t labels_offset, void *d_wire, uint64_t wire_bytes, void *stream) {
    if (bits_count < 1 || bits_count > 32 || bits_label < 1 || bits_label > 32 || !d_wire || !d_num_labels ||
        (n_rows && !d_offsets) || (cols_cap && !d_cols) || wire_bytes % 16 || labels_offset % 16 ||
        labels_offset < mbrwt_wire_labels_offset(n_rows, bits_count)) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    const uint64_t lab_off = labels_offset;
    const uint64_t lab_words = (labels_cap * bits_label + 31) / 32;
    if (lab_off + lab_words * 4 > wire_bytes) {
        set_error("wire segment too small for the rows and the label capacity");
        return MBRWT_ERR_INVALID;
    }
    const hipStream_t s = (hipStream_t)stream;
    // the pads and the unused label words are zero (the wire is deterministic)
    MBRWT_HIP(hipMemsetAsync(d_wire, 0, wire_bytes, s));
    // 32 values per thread = `bits` words; the fields' last chunks may run past
    // their words: the layout keeps room for whole chunks (checked below)
    const uint64_t cnt_chunks = (n_rows + 31) / 32, lab_chunks = (labels_cap + 31) / 32;
    if (8 + cnt_chunks * bits_count * 4 > lab_off || lab_off + lab_chunks * bits_label * 4 > wire_bytes) {
        set_error("wire segment too small for whole 32-value chunks");
        return MBRWT_ERR_INVALID;
    }
    const uint64_t cnt_words = (n_rows * bits_count + 31) / 32, lab_words_used = (labels_cap * bits_label + 31) / 32;
    hipLaunchKernelGGL(k_pack_csr, dim3(grid_of(std::max<uint64_t>(1, cnt_words + lab_words_used))), dim3(256), 0, s,
                       d_offsets, n_rows, d_cols, cols_cap, d_num_labels, labels_cap, bits_count, bits_label,
                       reinterpret_cast<uint32_t *>(d_wire), lab_off / 4, cnt_words, lab_words_used);
    MBRWT_HIP(hipGetLastError());
    return MBRWT_OK;
}

int mbrwt_unpack_labels_device(const void *d_base, uint32_t nseg, uint64_t seg_stride, uint64_t labels_offset,
                               uint64_t labels_cap, uint32_t bits, uint32_t *d_values, uint64_t values_cap,
                               uint64_t *d_status, void *stream) {
    if (bits < 1 || bits > 32 || !d_base || !d_status || nseg < 1 || nseg > kMaxSegs || seg_stride % 4 ||
        labels_offset % 4 || (values_cap && !d_values)) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    const uint64_t bound = std::min<uint64_t>(values_cap, (uint64_t)nseg * labels_cap);
    // one tile per workgroup (no grid-stride rounds: a workgroup's tile is
    // two dependent memory latencies, so rounds serialise them)
    const unsigned tiles = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((bound + kUnpackTile - 1) / kUnpackTile, 1u << 20));
    hipLaunchKernelGGL(k_unpack_labels_dev, dim3(tiles), dim3(256), 0,
                       (hipStream_t)stream, reinterpret_cast<const uint8_t *>(d_base), seg_stride, nseg, labels_offset,
                       labels_cap, bits, d_values, values_cap, reinterpret_cast<unsigned long long *>(d_status));
    MBRWT_HIP(hipGetLastError());
    return MBRWT_OK;
}

}  // extern "C"

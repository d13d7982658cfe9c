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

// k_pack_csr for 12-bit counts and labels (every BASELINE shape: < 4,096
// columns): thread t packs values 8 t .. 8 t + 7 of a field into its words
// 3 t .. 3 t + 2 (8 x 12 bits = 3 words exactly) -- 16-byte loads of the
// labels (or of the offsets), three word stores; a thread whose 8 values run
// past the field's end packs them one by one.  Threads [0, cnt_threads) pack
// the counts, the rest the labels.
__global__ __launch_bounds__(256) void k_pack_csr12(const uint64_t *__restrict__ offsets, uint64_t n_rows,
                                                    const uint32_t *__restrict__ cols, uint64_t cols_cap,
                                                    const uint64_t *__restrict__ num_labels, uint64_t cap,
                                                    uint32_t *__restrict__ wire, uint64_t lab_word0,
                                                    uint64_t cnt_threads, uint64_t lab_threads) {
    const uint64_t L = gld(num_labels);
    const bool lost = L > cols_cap;
    const uint64_t nl = lost ? 0 : L < cap ? L : cap;
    const uint64_t hdr = lost ? ~0ull : L;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        gst(wire, (uint32_t)hdr);
        gst(wire + 1, (uint32_t)(hdr >> 32));
    }
    if (lost) return;
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= cnt_threads + lab_threads) return;
    const bool lab = g >= cnt_threads;
    const uint64_t t = lab ? g - cnt_threads : g;
    const uint64_t n = lab ? nl : n_rows;
    const uint64_t i0 = 8 * t;
    if (i0 >= n) return;  // (the words past the field's values stay zero: memset)
    uint32_t v[8];
    if (i0 + 8 <= n) {
        if (lab) {
            const u32x4_t a = *(const AS_GLOBAL u32x4_t *)(uintptr_t)(cols + i0);
            const u32x4_t b = *(const AS_GLOBAL u32x4_t *)(uintptr_t)(cols + i0 + 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
            v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        } else {
            uint64_t o[9];
#pragma unroll
            for (uint32_t j = 0; j < 9; ++j) o[j] = gld(offsets + i0 + j);
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) v[j] = (uint32_t)(o[j + 1] - o[j]);
        }
    } else {
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
            const uint64_t i = i0 + j;
            v[j] = i < n ? (lab ? gld(cols + i) : (uint32_t)(gld(offsets + i + 1) - gld(offsets + i))) : 0u;
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) v[j] &= 0xFFFu;
    const uint32_t w0 = v[0] | (v[1] << 12) | (v[2] << 24);
    const uint32_t w1 = (v[2] >> 8) | (v[3] << 4) | (v[4] << 16) | (v[5] << 28);
    const uint32_t w2 = (v[5] >> 4) | (v[6] << 8) | (v[7] << 20);
    uint32_t *dst = wire + (lab ? lab_word0 : 2) + 3 * t;
    gst(dst, w0);
    gst(dst + 1, w1);
    gst(dst + 2, w2);
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

// The global offsets from the wire's packed row counts (at byte 8 of every
// segment): three passes over blocks of kOffRows rows -- per-block sums,
// one workgroup scanning the sums, then each block's counts re-read and
// scanned in LDS with the block's prefix added, written as coalesced u64s.
// (A hipcub scan over an iterator unpacking the counts took 87 us for 8 M
// rows: its per-item loads do not coalesce.)
constexpr uint32_t kWireScanSegs = 8;
constexpr uint32_t kOffRows = 2048;  // rows per block: 8 per thread
struct WireFirst {
    uint64_t v[kWireScanSegs + 1];
};
struct WireCounts {
    const uint8_t *base;
    uint64_t stride;
    uint32_t nseg, bits;
    WireFirst f;
};
// row i's count (i < N); first[] in LDS
__device__ __forceinline__ uint32_t wire_count(const WireCounts &w, const uint64_t *first, uint64_t i) {
    uint32_t sg = 0;
#pragma unroll
    for (uint32_t k = 1; k < kWireScanSegs; ++k) sg += (k < w.nseg && i >= first[k]) ? 1u : 0u;
    const uint32_t *p = reinterpret_cast<const uint32_t *>(w.base + sg * w.stride + 8);
    const uint64_t pos = (i - first[sg]) * w.bits;
    const uint64_t k = pos >> 5;
    const uint32_t off = (uint32_t)(pos & 31);
    uint32_t x = gld(p + k) >> off;
    if (off + w.bits > 32) x |= gld(p + k + 1) << (32 - off);
    return w.bits == 32 ? x : (x & ((1u << w.bits) - 1u));
}
__device__ __forceinline__ uint64_t block_sum256(uint64_t v, uint64_t *red) {
#pragma unroll
    for (uint32_t d = 32; d > 0; d >>= 1) v += __shfl_down(v, d, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    const uint64_t t = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    return t;
}
__global__ __launch_bounds__(256) void k_off_sums(WireCounts w, uint64_t *sums) {
    __shared__ uint64_t first[kWireScanSegs + 1];
    __shared__ uint64_t red[4];
    if (threadIdx.x <= kWireScanSegs) first[threadIdx.x] = w.f.v[threadIdx.x];
    __syncthreads();
    const uint64_t N = first[w.nseg];
    const uint64_t i0 = (uint64_t)blockIdx.x * kOffRows + 8 * threadIdx.x;  // (blocked: 16.5 vs 22 us striped)
    uint64_t s = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j)
        if (i0 + j < N) s += wire_count(w, first, i0 + j);
    const uint64_t t = block_sum256(s, red);
    if (threadIdx.x == 0) sums[blockIdx.x] = t;
}
// one workgroup: exclusive scan of the block sums in place, in chunks of 1,024
__global__ __launch_bounds__(1024) void k_off_scan_sums(uint64_t *sums, uint64_t nblk) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint64_t c0 = 0; c0 < nblk; c0 += 1024) {
        const uint64_t i = c0 + threadIdx.x;
        const uint64_t v = i < nblk ? sums[i] : 0;
        uint64_t x = v;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        if (lane == 63) wsum[wv] = x;
        __syncthreads();
        uint64_t before = carry;
        for (uint32_t k = 0; k < wv; ++k) before += wsum[k];
        if (i < nblk) sums[i] = before + x - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry = before + x;
        __syncthreads();
    }
}
// counts loaded and offsets stored row-striped (row base + t + 256 j:
// coalesced), scanned blocked (thread t: rows 8 t .. 8 t + 7) through LDS
__global__ __launch_bounds__(256) void k_off_write(WireCounts w, const uint64_t *sums, uint64_t *offsets) {
    __shared__ uint64_t first[kWireScanSegs + 1];
    __shared__ uint64_t wsum[4];
    // counts, then block-relative inclusive prefixes: u64, as k_off_sums' block
    // sums -- 2,048 counts of up to 32 bits can pass 2^32
    __shared__ uint64_t lc[kOffRows];
    if (threadIdx.x <= kWireScanSegs) first[threadIdx.x] = w.f.v[threadIdx.x];
    __syncthreads();
    const uint64_t N = first[w.nseg];
    const uint64_t rb = (uint64_t)blockIdx.x * kOffRows;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        const uint64_t i = rb + threadIdx.x + 256 * j;
        lc[threadIdx.x + 256 * j] = i < N ? wire_count(w, first, i) : 0u;
    }
    __syncthreads();
    uint64_t c[8], s = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        c[j] = lc[8 * threadIdx.x + j];
        s += c[j];
    }
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t x = s;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint64_t run = x - s;
    for (uint32_t k = 0; k < wv; ++k) run += wsum[k];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        run += c[j];
        lc[8 * threadIdx.x + j] = run;
    }
    __syncthreads();
    const uint64_t base = sums[blockIdx.x];
    if (blockIdx.x == 0 && threadIdx.x == 0) offsets[0] = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t r = threadIdx.x + 256 * j;
        if (rb + r < N) offsets[rb + r + 1] = base + lc[r];
    }
}

// labels of <= 12 bits (every BASELINE shape: < 4,096 columns): thread t of
// a workgroup takes labels 8 t .. 8 t + 7 of each of the workgroup's R tiles
// of 2,048 -- one 16-byte load covers their <= 96 bits (plus the offset
// into the first word), two 16-byte stores write them; every load of the
// workgroup is issued before its first store (the headers' latency is paid
// once per R tiles, not per tile), no LDS stage.  A group of 8 that crosses
// a segment boundary takes the label-by-label path.
constexpr uint32_t kUnpackTiles12 = 4;
__global__ __launch_bounds__(256) void k_unpack_labels12(const uint8_t *__restrict__ base, uint64_t stride,
                                                         uint32_t nseg, uint64_t lab_off, uint64_t cap,
                                                         uint32_t bits, uint32_t *__restrict__ out,
                                                         uint64_t out_cap, unsigned long long *status) {
    __shared__ uint64_t first[kMaxSegs + 1];
    __shared__ uint32_t bad;
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
    const uint32_t mask = (1u << bits) - 1u;
    auto seg_of = [&](uint64_t i) {
        uint32_t lo = 0, hi = nseg;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (first[mid] <= i) lo = mid;
            else hi = mid;
        }
        return lo;
    };
    u32x4_t v[kUnpackTiles12];
    uint32_t sh[kUnpackTiles12];
    bool fast[kUnpackTiles12];
    const uint64_t seg_words = (cap + 31) / 32 * bits;  // a segment's label words (whole 32-value chunks)
    const uint64_t g0 = (uint64_t)blockIdx.x * kUnpackTiles12 * kUnpackTile;
#pragma unroll
    for (uint32_t r = 0; r < kUnpackTiles12; ++r) {
        const uint64_t i = g0 + (uint64_t)r * kUnpackTile + 8 * threadIdx.x;
        fast[r] = false;
        sh[r] = 0;
        if (i >= N) continue;
        const uint32_t sg = seg_of(i);
        if (i + 8 > first[sg + 1]) continue;  // (crosses a segment's end, or the batch's: slow path)
        const uint64_t pos = (i - first[sg]) * bits;
        if ((pos >> 5) + 4 > seg_words) continue;  // (the 4 words must lie in the segment's label words)
        const uint32_t *w = reinterpret_cast<const uint32_t *>(base + sg * stride + lab_off) + (pos >> 5);
        sh[r] = (uint32_t)(pos & 31);
        v[r] = u32x4_t{gld(w), gld(w + 1), gld(w + 2), gld(w + 3)};
        fast[r] = true;
    }
#pragma unroll
    for (uint32_t r = 0; r < kUnpackTiles12; ++r) {
        const uint64_t i = g0 + (uint64_t)r * kUnpackTile + 8 * threadIdx.x;
        if (i >= N) continue;
        if (fast[r]) {
            const uint64_t lo = (uint64_t)v[r].x | ((uint64_t)v[r].y << 32);
            const uint64_t hi = (uint64_t)v[r].z | ((uint64_t)v[r].w << 32);
            // bits [sh, sh + 8 bits) of the 128-bit value hi:lo
            uint32_t lab[8];
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t b = sh[r] + j * bits;  // < 128
                const uint64_t a = b < 64 ? (lo >> b) | (b ? hi << (64 - b) : 0) : hi >> (b - 64);
                lab[j] = (uint32_t)a & mask;
            }
            u32x4_t o0{lab[0], lab[1], lab[2], lab[3]}, o1{lab[4], lab[5], lab[6], lab[7]};
            *(AS_GLOBAL u32x4_t *)(uintptr_t)(out + i) = o0;
            *(AS_GLOBAL u32x4_t *)(uintptr_t)(out + i + 4) = o1;
        } else {
            const uint64_t e = i + 8 < N ? i + 8 : N;
            for (uint64_t k = i; k < e; ++k) {
                const uint32_t sg = seg_of(k);
                const uint32_t *wd = reinterpret_cast<const uint32_t *>(base + sg * stride + lab_off);
                const uint64_t pos = (k - first[sg]) * bits;
                const uint64_t w = pos >> 5;
                const uint32_t off = (uint32_t)(pos & 31);
                uint32_t x = gld(wd + w) >> off;
                if (off + bits > 32) x |= gld(wd + w + 1) << (32 - off);
                gst(out + k, x & mask);
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
    if (bits_count == 12 && bits_label == 12 && (reinterpret_cast<uintptr_t>(d_cols) & 15) == 0 && lab_off % 4 == 0) {
        // (16-byte label loads at value 8 t: the CSR must be 16-byte aligned)
        const uint64_t ct = (n_rows + 7) / 8, lt = (labels_cap + 7) / 8;
        const uint64_t th = std::max<uint64_t>(1, ct + lt);
        if ((th + 255) / 256 > 0x7FFFFFFFull) {
            set_error("batch too large for the pack grid");
            return MBRWT_ERR_UNSUPPORTED;
        }
        hipLaunchKernelGGL(k_pack_csr12, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, s, d_offsets, n_rows, d_cols,
                           cols_cap, d_num_labels, labels_cap, reinterpret_cast<uint32_t *>(d_wire), lab_off / 4, ct, lt);
        MBRWT_HIP(hipGetLastError());
        return MBRWT_OK;
    }
    const uint64_t cnt_words = (n_rows * bits_count + 31) / 32, lab_words_used = (labels_cap * bits_label + 31) / 32;
    hipLaunchKernelGGL(k_pack_csr, dim3(grid_of(std::max<uint64_t>(1, cnt_words + lab_words_used))), dim3(256), 0, s,
                       d_offsets, n_rows, d_cols, cols_cap, d_num_labels, labels_cap, bits_count, bits_label,
                       reinterpret_cast<uint32_t *>(d_wire), lab_off / 4, cnt_words, lab_words_used);
    MBRWT_HIP(hipGetLastError());
    return MBRWT_OK;
}

int mbrwt_unpack_offsets_device(const void *d_base, uint32_t nseg, uint64_t seg_stride, const uint64_t *counts,
                                uint32_t bits, uint64_t *d_offsets, void *d_temp, uint64_t *temp_bytes,
                                void *stream) {
    if (bits < 1 || bits > 32 || !d_base || !counts || !temp_bytes || nseg < 1 || seg_stride % 4 ||
        (d_temp && !d_offsets)) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    if (nseg > kWireScanSegs) {
        set_error("more than 8 segments: unpack the counts (mbrwt_unpack_segments_device) and scan them");
        return MBRWT_ERR_UNSUPPORTED;
    }
    WireCounts wc{reinterpret_cast<const uint8_t *>(d_base), seg_stride, nseg, bits, WireFirst{}};
    for (uint32_t r = 0; r < nseg; ++r) wc.f.v[r + 1] = wc.f.v[r] + counts[r];
    for (uint32_t r = nseg + 1; r <= kWireScanSegs; ++r) wc.f.v[r] = wc.f.v[nseg];
    const uint64_t N = wc.f.v[nseg];
    const uint64_t nblk = (N + kOffRows - 1) / kOffRows;
    // scratch: the block sums
    const uint64_t need = std::max<uint64_t>(1, nblk) * 8;
    if (!d_temp) {
        *temp_bytes = need;
        return MBRWT_OK;
    }
    if (*temp_bytes < need) {
        set_error("scratch smaller than the size the scan needs");
        return MBRWT_ERR_INVALID;
    }
    if (nblk > 0x7FFFFFFFull) {
        set_error("too many rows");
        return MBRWT_ERR_UNSUPPORTED;
    }
    const hipStream_t s = (hipStream_t)stream;
    if (!N) {
        MBRWT_HIP(hipMemsetAsync(d_offsets, 0, 8, s));
        return MBRWT_OK;
    }
    uint64_t *sums = reinterpret_cast<uint64_t *>(d_temp);
    hipLaunchKernelGGL(k_off_sums, dim3((unsigned)nblk), dim3(256), 0, s, wc, sums);
    MBRWT_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_off_scan_sums, dim3(1), dim3(1024), 0, s, sums, nblk);
    MBRWT_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_off_write, dim3((unsigned)nblk), dim3(256), 0, s, wc, (const uint64_t *)sums, d_offsets);
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
    if (bits <= 12 && (reinterpret_cast<uintptr_t>(d_values) & 15) == 0) {
        // (16-byte stores at label 8 t: the output must be 16-byte aligned)
        const uint64_t per = (uint64_t)kUnpackTiles12 * kUnpackTile;
        const unsigned wgs = (unsigned)std::max<uint64_t>(1, (bound + per - 1) / per);
        if ((bound + per - 1) / per > (1u << 24)) {
            set_error("batch too large for the unpack grid");
            return MBRWT_ERR_UNSUPPORTED;
        }
        hipLaunchKernelGGL(k_unpack_labels12, dim3(wgs), dim3(256), 0, (hipStream_t)stream,
                           reinterpret_cast<const uint8_t *>(d_base), seg_stride, nseg, labels_offset, labels_cap, bits,
                           d_values, values_cap, reinterpret_cast<unsigned long long *>(d_status));
        MBRWT_HIP(hipGetLastError());
        return MBRWT_OK;
    }
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

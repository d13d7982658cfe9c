// binrel_wt.hip -- BinRel-WT on the device (reference
// annotation/bin_rel_wt/bin_rel_wt_sdsl.cpp, an sdsl::wt_int over the
// concatenated rows plus a delimiter bit vector).
//
// Device layout (MI355X-first, result-identical to the reference):
// * The row delimiters become the CSR offsets they encode:
//   select1(row + 1) - row == offsets[row] (bin_rel_wt_sdsl.cpp:58-62), kept
//   as a u64 array in HBM (one 16-byte read per row instead of two selects).
// * The string of column ids is held in a 4-ARY WAVELET MATRIX (not the
//   binary levelwise wavelet tree of wt_int): level l stores the 2-bit digit
//   l (from the top) of every symbol, the symbols of level l+1 being level
//   l's stably partitioned by that digit into 4 buckets; a position maps
//   down with ONE rank per level (digit d: Z_l[d] + rank_d(p)), so decoding
//   needs no node boundaries and ceil(w/2) levels instead of w (6 instead of
//   12 at 3,173 columns): half the dependent random block reads per label.
// * Rows are stored with their ids ascending.  That changes no query result
//   (get_row returns the ascending distinct ids, get is membership,
//   get_column lists rows in row order) and makes a row's decoded positions
//   come out in output order: get_row is "access" of the row's contiguous
//   string range, one thread per output label, with adjacent threads walking
//   adjacent positions (their level reads coalesce).
// * Every level is a sequence of 64-byte rank blocks {u32 occurrences of
//   digits 0, 1, 2 before the block, 13 u32 words of 16 digits} = 208
//   positions; a rank is one 64-byte segment (the 16-byte quarters up to the
//   position's word) plus popcounts of digit-match masks.
// * Rows are cut into chunks of 2^k rows with < 2^31 symbols each (u32
//   positions and ranks), each chunk an independent wavelet matrix.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/mbrwt_wt.h"
#include "device_access.hpp"
#include "mbrwt_internal.hpp"

namespace mbrwt {
namespace {

constexpr uint32_t kWtBlockPos = 208;    // 2-bit digits per 64-byte rank block
constexpr uint32_t kWtBlockBytes = 64;
constexpr uint32_t kWtMaxLevels = 16;    // digit levels (symbols of <= 32 bits)

struct WtChunkDev {
    uint64_t base;       // level 0 block array; level l at base + l * level_bytes
    uint64_t str0;       // global string offset of the chunk's first symbol
    uint64_t level_bytes;
    uint32_t len;        // symbols in the chunk
    uint32_t pad;
    uint32_t z[kWtMaxLevels][4];  // level l: start of digit v's bucket in level l + 1
};

__device__ __forceinline__ uint64_t mix64_d(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// bit 2i of the result is set iff digit i of x equals the digit in pat
// (pat = digit * 0x55555555)
__device__ __forceinline__ uint32_t digit_matches(uint32_t x, uint32_t pat) {
    const uint32_t y = x ^ pat;
    return ~(y | (y >> 1)) & 0x55555555u;
}

// A level's block at `a`: dwords 0..2 = digits 0, 1, 2 before the block;
// dwords 3..15 = 13 words of 16 digits (digit i of word k = position 16k + i).
// The words up to word k are read (1..4 16-byte loads of one 64-byte segment).
struct WtBlock {
    uint32_t c0, c1, c2;
    uint32_t w[13];
    __device__ __forceinline__ void load(uint64_t a, uint32_t k) {
        const uint4 q0 = gld_at<uint4>(a);
        c0 = q0.x;
        c1 = q0.y;
        c2 = q0.z;
        w[0] = q0.w;
#pragma unroll
        for (uint32_t h = 1; h < 4; ++h) {
            if (k >= 4 * h - 3) {
                const uint4 q = gld_at<uint4>(a + 16 * h);
                w[4 * h - 3] = q.x;
                w[4 * h - 2] = q.y;
                w[4 * h - 1] = q.z;
                w[4 * h] = q.w;
            } else {
                w[4 * h - 3] = w[4 * h - 2] = w[4 * h - 1] = w[4 * h] = 0;
            }
        }
    }
    __device__ __forceinline__ uint32_t before(uint32_t blk, uint32_t v) const {
        return v == 0 ? c0 : v == 1 ? c1 : v == 2 ? c2 : blk * kWtBlockPos - c0 - c1 - c2;
    }
    // occurrences of digit v in positions [0, 16k + b) of the block
    __device__ __forceinline__ uint32_t count(uint32_t v, uint32_t k, uint32_t b) const {
        const uint32_t pat = v * 0x55555555u;
        uint32_t r = 0, x = 0;
#pragma unroll
        for (uint32_t i = 0; i < 13; ++i) {
            const uint32_t m = digit_matches(w[i], pat);
            if (i < k) r += __builtin_popcount(m);
            x = i == k ? m : x;
        }
        return r + __builtin_popcount(x & ((1u << (2 * b)) - 1u));
    }
};

// rank of digit v at position p of a level: occurrences in [0, p)
__device__ __forceinline__ uint32_t wt_rank(uint64_t lvl, uint32_t p, uint32_t v) {
    const uint32_t blk = p / kWtBlockPos, o = p - blk * kWtBlockPos;
    WtBlock B;
    B.load(lvl + (uint64_t)blk * kWtBlockBytes, o >> 4);
    return B.before(blk, v) + B.count(v, o >> 4, o & 15);
}

// access + rank: digit d at position p, returns occurrences of d in [0, p)
__device__ __forceinline__ uint32_t wt_access_rank(uint64_t lvl, uint32_t p, uint32_t &d) {
    const uint32_t blk = p / kWtBlockPos, o = p - blk * kWtBlockPos, k = o >> 4, b = o & 15;
    WtBlock B;
    B.load(lvl + (uint64_t)blk * kWtBlockBytes, k);
    uint32_t wk = B.w[0];
#pragma unroll
    for (uint32_t i = 1; i < 13; ++i) wk = i == k ? B.w[i] : wk;
    d = (wk >> (2 * b)) & 3u;
    return B.before(blk, d) + B.count(d, k, b);
}

// position of the j-th (1-based) occurrence of digit v in a level of nblk1
// blocks (the last one the sentinel)
__device__ uint32_t wt_select(uint64_t lvl, uint32_t nblk1, uint32_t v, uint32_t j) {
    uint32_t lo = 0, hi = nblk1;  // last block with occurrences before it < j
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint4 q = gld_at<uint4>(lvl + (uint64_t)mid * kWtBlockBytes);
        const uint32_t before = v == 0 ? q.x : v == 1 ? q.y : v == 2 ? q.z : mid * kWtBlockPos - q.x - q.y - q.z;
        if (before < j) lo = mid;
        else hi = mid;
    }
    WtBlock B;
    B.load(lvl + (uint64_t)lo * kWtBlockBytes, 12);
    uint32_t need = j - B.before(lo, v);
    const uint32_t pat = v * 0x55555555u;
    for (uint32_t k = 0; k < 13; ++k) {
        uint32_t m = digit_matches(B.w[k], pat);
        const uint32_t c = __builtin_popcount(m);
        if (need <= c) {
            while (--need) m &= m - 1;
            return lo * kWtBlockPos + 16 * k + (__builtin_ctz(m) >> 1);
        }
        need -= c;
    }
    return 0xFFFFFFFFu;  // not reached for valid j
}

// ---- construction ----------------------------------------------------------

// one word of 16 digits (bits sh, sh+1 of the symbols)
__global__ void k_wt_words(const uint32_t *__restrict__ sym, uint64_t len, uint32_t sh, uint32_t *__restrict__ words,
                           uint64_t nwords) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += gstride) {
        uint32_t x = 0;
        const uint64_t p0 = 16 * w;
        for (uint32_t k = 0; k < 16 && p0 + k < len; ++k) x |= ((sym[p0 + k] >> sh) & 3u) << (2 * k);
        words[w] = x;
    }
}

// digits 0, 1, 2 per block (positions >= len, padded with digit 0, excluded):
// cnt[v * stride + b]
__global__ void k_wt_block_counts(const uint32_t *__restrict__ words, uint64_t nwords, uint64_t len,
                                  uint32_t *__restrict__ cnt, uint64_t stride, uint64_t nblk) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nblk; b += gstride) {
        uint32_t c[3] = {0, 0, 0};
        for (uint32_t k = 0; k < 13; ++k) {
            const uint64_t wi = 13 * b + k;
            if (wi >= nwords) break;
            const uint64_t valid = len - 16 * wi;  // > 0
            const uint32_t keep = valid >= 16 ? 0x55555555u : 0x55555555u & ((1u << (2 * valid)) - 1u);
            for (uint32_t v = 0; v < 3; ++v) c[v] += __builtin_popcount(digit_matches(words[wi], v * 0x55555555u) & keep);
        }
        for (uint32_t v = 0; v < 3; ++v) cnt[v * stride + b] = c[v];
    }
}

// blocks [0, nblk) + the sentinel block nblk (counts = totals, zero words)
__global__ void k_wt_blocks(const uint32_t *__restrict__ words, uint64_t nwords, const uint32_t *__restrict__ ranks,
                            uint64_t stride, uint64_t nblk, uint32_t *__restrict__ out) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b <= nblk; b += gstride) {
        uint32_t *o = out + 16 * b;
        for (uint32_t v = 0; v < 3; ++v) o[v] = ranks[v * stride + b];
        for (uint32_t k = 0; k < 13; ++k) o[3 + k] = (b < nblk && 13 * b + k < nwords) ? words[13 * b + k] : 0u;
    }
}

// synthetic rows: per-row counts / ascending ids (thread per row)
__global__ void k_wt_synth_count(uint64_t row0, uint64_t nrows, uint32_t num_columns, uint64_t T, uint64_t seed,
                                 uint32_t *__restrict__ cnt) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrows; i += gstride) {
        const uint64_t K = mix64_d(seed ^ ((row0 + i + 1) * 0x9E3779B97F4A7C15ull));
        uint32_t c = 0;
        for (uint32_t col = 0; col < num_columns; ++col)
            c += (T == ~0ull || mix64_d(K + col * 0xD1B54A32D192ED03ull) < T) ? 1u : 0u;
        cnt[i] = c;
    }
}

__global__ void k_wt_synth_write(uint64_t row0, uint64_t nrows, uint32_t num_columns, uint64_t T, uint64_t seed,
                                 const uint32_t *__restrict__ off, uint64_t str0, uint32_t *__restrict__ sym,
                                 uint64_t *__restrict__ goff) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrows; i += gstride) {
        const uint64_t K = mix64_d(seed ^ ((row0 + i + 1) * 0x9E3779B97F4A7C15ull));
        uint32_t o = off[i];
        goff[row0 + i] = str0 + o;
        for (uint32_t col = 0; col < num_columns; ++col)
            if (T == ~0ull || mix64_d(K + col * 0xD1B54A32D192ED03ull) < T) sym[o++] = col;
    }
}

// ---- queries ---------------------------------------------------------------

struct WtParams {
    const WtChunkDev *chunks;
    const uint64_t *offsets;  // [num_rows + 1] global string offsets
    uint64_t num_rows, num_columns;
    uint32_t w, log2_rows;  // symbol bits; rows per chunk = 2^log2_rows
    uint32_t levels;        // 2-bit digit levels = ceil(w / 2)
    unsigned long long *scalars;  // [2] error flags
};

__global__ void k_wt_lengths(WtParams P, const uint64_t *__restrict__ rows, uint64_t n, uint64_t *__restrict__ lens) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        const uint64_t r = rows[i];
        if (r >= P.num_rows) {
            atomicOr(&P.scalars[2], 1ull);
            lens[i] = 0;
            continue;
        }
        lens[i] = P.offsets[r + 1] - P.offsets[r];
    }
}

constexpr int kWtTile = 256;

// get_row: one thread per output label of a 256-row tile of the batch
__global__ __launch_bounds__(kWtTile) void k_wt_decode(WtParams P, const uint64_t *__restrict__ rows, uint64_t n,
                                                       const uint64_t *__restrict__ csr, uint32_t *__restrict__ cols) {
    __shared__ uint64_t s_csr[kWtTile + 1];
    __shared__ uint64_t s_row[kWtTile];
    const uint32_t t = threadIdx.x;
    for (uint64_t tile = blockIdx.x; tile * kWtTile < n; tile += gridDim.x) {
        const uint64_t r0 = tile * kWtTile;
        const uint32_t rn = (uint32_t)(n - r0 < kWtTile ? n - r0 : kWtTile);
        for (uint32_t i = t; i <= rn; i += kWtTile) s_csr[i] = csr[r0 + i];
        for (uint32_t i = t; i < rn; i += kWtTile) s_row[i] = rows[r0 + i];
        __syncthreads();
        const uint64_t e0 = s_csr[0], e1 = s_csr[rn];
        for (uint64_t e = e0 + t; e < e1; e += kWtTile) {
            uint32_t lo = 0, hi = rn;  // last i with s_csr[i] <= e
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_csr[mid] <= e) lo = mid;
                else hi = mid;
            }
            const uint64_t row = s_row[lo];
            const WtChunkDev *ch = P.chunks + (row >> P.log2_rows);
            const uint64_t base = ch->base, lb = ch->level_bytes;
            uint32_t p = (uint32_t)(P.offsets[row] + (e - s_csr[lo]) - ch->str0);
            uint32_t sym = 0;
            for (uint32_t l = 0; l < P.levels; ++l) {
                uint32_t d;
                const uint32_t r = wt_access_rank(base + l * lb, p, d);
                sym = (sym << 2) | d;
                p = ch->z[l][d] + r;
            }
            cols[e] = sym;
        }
        __syncthreads();
    }
}

// get(row, col): rank difference of col over the row's range
__global__ void k_wt_get(WtParams P, const uint64_t *__restrict__ rows, const uint64_t *__restrict__ qcols,
                         uint64_t n, uint8_t *__restrict__ out) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        const uint64_t row = rows[i], col = qcols[i];
        if (row >= P.num_rows || col >= P.num_columns) {
            atomicOr(&P.scalars[2], 1ull);
            out[i] = 0;
            continue;
        }
        const WtChunkDev *ch = P.chunks + (row >> P.log2_rows);
        uint32_t s = (uint32_t)(P.offsets[row] - ch->str0), e = (uint32_t)(P.offsets[row + 1] - ch->str0);
        for (uint32_t l = 0; l < P.levels && s < e; ++l) {
            const uint64_t lvl = ch->base + l * ch->level_bytes;
            const uint32_t d = (uint32_t)(col >> (2 * (P.levels - 1 - l))) & 3u;
            s = ch->z[l][d] + wt_rank(lvl, s, d);
            e = ch->z[l][d] + wt_rank(lvl, e, d);
        }
        out[i] = e > s ? 1 : 0;
    }
}

// get_column, pass 1: per chunk, the bottom-level range of the column
__global__ void k_wt_col_range(WtParams P, uint64_t nchunks, uint32_t col, uint32_t *__restrict__ start,
                               uint64_t *__restrict__ count) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks; c += gstride) {
        const WtChunkDev *ch = P.chunks + c;
        uint32_t s = 0, e = ch->len;
        for (uint32_t l = 0; l < P.levels && s < e; ++l) {
            const uint64_t lvl = ch->base + l * ch->level_bytes;
            const uint32_t d = (col >> (2 * (P.levels - 1 - l))) & 3u;
            s = ch->z[l][d] + wt_rank(lvl, s, d);
            e = ch->z[l][d] + wt_rank(lvl, e, d);
        }
        start[c] = s;
        count[c] = e > s ? e - s : 0;
    }
}

// get_column, pass 2: lift every occurrence to the top level (selects) and
// map its string position to the row (binary search over the chunk's offsets)
__global__ void k_wt_col_lift(WtParams P, uint64_t nchunks, uint32_t col, const uint32_t *__restrict__ start,
                              const uint64_t *__restrict__ coff, uint64_t total, uint64_t *__restrict__ out) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gstride) {
        uint64_t lo = 0, hi = nchunks;  // last chunk with coff <= i
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (coff[mid] <= i) lo = mid;
            else hi = mid;
        }
        const WtChunkDev *ch = P.chunks + lo;
        const uint32_t nblk1 = (uint32_t)(ch->level_bytes / kWtBlockBytes);
        uint32_t q = start[lo] + (uint32_t)(i - coff[lo]);
        for (uint32_t l = P.levels; l-- > 0;) {
            const uint64_t lvl = ch->base + l * ch->level_bytes;
            const uint32_t d = (col >> (2 * (P.levels - 1 - l))) & 3u;
            q = wt_select(lvl, nblk1, d, q - ch->z[l][d] + 1);
        }
        // row = last row of the chunk whose start offset <= str0 + q
        const uint64_t g = ch->str0 + q;
        uint64_t rlo = lo << P.log2_rows, rhi = std::min<uint64_t>((lo + 1) << P.log2_rows, P.num_rows);
        while (rhi - rlo > 1) {
            const uint64_t mid = (rlo + rhi) >> 1;
            if (P.offsets[mid] <= g) rlo = mid;
            else rhi = mid;
        }
        out[i] = rlo;
    }
}

unsigned grid_for(uint64_t n, unsigned per = 256) {
    const uint64_t g = (n + per - 1) / per;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, 1u << 20));
}

}  // namespace

// ---- context ---------------------------------------------------------------

struct WtCtx {
    int device = 0;
    uint64_t num_rows = 0, num_columns = 0, num_relations = 0;
    uint32_t w = 1, log2_rows = 20;
    std::vector<WtChunkDev> chunks;
    std::vector<void *> allocs;
    uint64_t *d_offsets = nullptr;
    WtChunkDev *d_chunks = nullptr;
    uint64_t device_bytes = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    WsFenceState fence;  // orders workspace use across callers' streams (mbrwt_internal.hpp)
    Workspace ws_a, ws_b, ws_c, ws_scan, ws_io;
    Workspace ws_cls_off, ws_cls_cols, ws_cls_cnt;  // classify: the rows' CSR, per-read counts
    uint64_t *h_scalars = nullptr, *d_scalars = nullptr;
    bool timing = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double timing_ms = 0;
    uint64_t timing_launches = 0;

    WtParams params() const {
        WtParams p;
        p.chunks = d_chunks;
        p.offsets = d_offsets;
        p.num_rows = num_rows;
        p.num_columns = num_columns;
        p.w = w;
        p.levels = (w + 1) / 2;
        p.log2_rows = log2_rows;
        p.scalars = reinterpret_cast<unsigned long long *>(d_scalars);
        return p;
    }
    ~WtCtx() {
        for (void *a : allocs) (void)hipFree(a);
        if (d_offsets) (void)hipFree(d_offsets);
        if (d_chunks) (void)hipFree(d_chunks);
        for (Workspace *ws : {&ws_a, &ws_b, &ws_c, &ws_scan, &ws_io, &ws_cls_off, &ws_cls_cols, &ws_cls_cnt})
            if (ws->buf) (void)hipFree(ws->buf);
        if (h_scalars) (void)hipHostFree(h_scalars);
        if (d_scalars) (void)hipFree(d_scalars);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        destroy_fence(fence);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace {

uint32_t symbol_bits(uint64_t num_columns) {  // ids < num_columns
    uint32_t w = 1;
    while (w < 32 && (1ull << w) < num_columns) ++w;
    return w;
}

// Build the wavelet matrix of one chunk from its symbols (d_sym, len, in
// string order); d_sym and d_alt are consumed (sorted level by level).
int build_chunk(WtCtx &c, WtChunkDev &ch, uint32_t *d_sym, uint32_t *d_alt, uint64_t len, hipStream_t s) {
    const uint32_t levels = (c.w + 1) / 2;
    const uint64_t nwords = (len + 15) / 16, nblk = (len + kWtBlockPos - 1) / kWtBlockPos;
    const uint64_t stride = nblk + 2;  // per-digit count / rank arrays
    ch.len = (uint32_t)len;
    ch.level_bytes = (nblk + 1) * kWtBlockBytes;
    void *lv = nullptr;
    MBRWT_HIP(hipMalloc(&lv, ch.level_bytes * levels));
    c.allocs.push_back(lv);
    c.device_bytes += ch.level_bytes * levels;
    ch.base = reinterpret_cast<uint64_t>(lv);
    int rc;
    // workspace: words | 3 x block counts | 3 x ranks | totals | scan/sort temp
    size_t scan_bytes = 0, sort_bytes = 0;
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                               (int)(nblk + 1), s));
    MBRWT_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, sort_bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                                (int)std::max<uint64_t>(len, 1), 0, 2, s));
    if ((rc = ensure(c.ws_c, (nwords + 6 * stride + 4 * kWtMaxLevels) * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(c.ws_scan, std::max(scan_bytes, sort_bytes) + 16))) return rc;
    uint32_t *d_words = reinterpret_cast<uint32_t *>(c.ws_c.buf);
    uint32_t *d_cnt = d_words + nwords;
    uint32_t *d_rank = d_cnt + 3 * stride;
    uint32_t *d_tot = d_rank + 3 * stride;  // digits 0..2 per level, read back once
    for (uint32_t l = 0; l < levels; ++l) {
        const uint32_t sh = 2 * (levels - 1 - l);
        uint32_t *out = reinterpret_cast<uint32_t *>(ch.base + l * ch.level_bytes);
        if (nwords) {
            hipLaunchKernelGGL(k_wt_words, dim3(grid_for(nwords)), dim3(256), 0, s, d_sym, len, sh, d_words, nwords);
            hipLaunchKernelGGL(k_wt_block_counts, dim3(grid_for(nblk)), dim3(256), 0, s, d_words, nwords, len, d_cnt,
                               stride, nblk);
        }
        for (uint32_t v = 0; v < 3; ++v) {
            MBRWT_HIP(hipMemsetAsync(d_cnt + v * stride + nblk, 0, sizeof(uint32_t), s));
            MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(c.ws_scan.buf, scan_bytes, d_cnt + v * stride,
                                                       d_rank + v * stride, (int)(nblk + 1), s));
            MBRWT_HIP(hipMemcpyAsync(d_tot + 3 * l + v, d_rank + v * stride + nblk, sizeof(uint32_t),
                                     hipMemcpyDeviceToDevice, s));
        }
        hipLaunchKernelGGL(k_wt_blocks, dim3(grid_for(nblk + 1)), dim3(256), 0, s, d_words, nwords, d_rank, stride,
                           nblk, out);
        MBRWT_HIP(hipGetLastError());
        if (l + 1 < levels && len) {  // stable partition by this digit = one 2-bit radix pass
            MBRWT_HIP(hipcub::DeviceRadixSort::SortKeys(c.ws_scan.buf, sort_bytes, d_sym, d_alt, (int)len, (int)sh,
                                                        (int)sh + 2, s));
            std::swap(d_sym, d_alt);
        }
    }
    uint32_t tot[3 * kWtMaxLevels];
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, d_tot, 3 * levels * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    std::memcpy(tot, c.h_scalars, 3 * levels * sizeof(uint32_t));
    for (uint32_t l = 0; l < levels; ++l) {
        ch.z[l][0] = 0;
        ch.z[l][1] = tot[3 * l];
        ch.z[l][2] = tot[3 * l] + tot[3 * l + 1];
        ch.z[l][3] = tot[3 * l] + tot[3 * l + 1] + tot[3 * l + 2];
    }
    return MBRWT_OK;
}

int init_common(WtCtx &c, int device, uint64_t num_rows, uint64_t num_columns) {
    c.device = device;
    MBRWT_HIP(hipSetDevice(device));
    MBRWT_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    MBRWT_HIP(hipHostMalloc(reinterpret_cast<void **>(&c.h_scalars), 32 * sizeof(uint64_t)));
    MBRWT_HIP(hipMalloc(&c.d_scalars, 8 * sizeof(uint64_t)));
    MBRWT_HIP(hipEventCreate(&c.ev0));
    MBRWT_HIP(hipEventCreate(&c.ev1));
    MBRWT_HIP(create_fence(c.fence));
    c.num_rows = num_rows;
    c.num_columns = num_columns;
    c.w = symbol_bits(num_columns);
    // rows per chunk: a power of two with rows * num_columns < 2^31 (u32
    // positions and int item counts even for all-ones rows), at most 2^24
    uint32_t k = 24;
    while (k > 0 && ((1ull << k) * std::max<uint64_t>(num_columns, 1)) >= (1ull << 31)) --k;
    c.log2_rows = k;
    const uint64_t nch = num_rows ? ((num_rows - 1) >> k) + 1 : 0;
    c.chunks.assign(nch, WtChunkDev{});
    MBRWT_HIP(hipMalloc(reinterpret_cast<void **>(&c.d_offsets), (num_rows + 1) * sizeof(uint64_t)));
    c.device_bytes = (num_rows + 1) * sizeof(uint64_t);
    return MBRWT_OK;
}

int finish(WtCtx &c) {
    if (!c.chunks.empty()) {
        MBRWT_HIP(hipMalloc(reinterpret_cast<void **>(&c.d_chunks), c.chunks.size() * sizeof(WtChunkDev)));
        MBRWT_HIP(hipMemcpy(c.d_chunks, c.chunks.data(), c.chunks.size() * sizeof(WtChunkDev), hipMemcpyHostToDevice));
    }
    MBRWT_HIP(hipStreamSynchronize(c.stream));
    return MBRWT_OK;
}

int build_from_csr(WtCtx &c, const mbrwt_binrel_desc &d) {
    if (d.num_rows && (!d.offsets || (d.offsets[d.num_rows] && !d.cols))) {
        set_error("null offsets/cols");
        return MBRWT_ERR_INVALID;
    }
    if (d.num_rows && d.offsets[0] != 0) {
        set_error("offsets[0] != 0");
        return MBRWT_ERR_INVALID;
    }
    for (uint64_t r = 0; r < d.num_rows; ++r)
        if (d.offsets[r + 1] < d.offsets[r]) {
            set_error("offsets not monotone");
            return MBRWT_ERR_INVALID;
        }
    int rc = init_common(c, c.device, d.num_rows, d.num_columns);
    if (rc) return rc;
    c.num_relations = d.num_rows ? d.offsets[d.num_rows] : 0;
    if (d.num_rows) {
        MBRWT_HIP(hipMemcpy(c.d_offsets, d.offsets, (d.num_rows + 1) * sizeof(uint64_t), hipMemcpyHostToDevice));
    } else {
        MBRWT_HIP(hipMemset(c.d_offsets, 0, sizeof(uint64_t)));
    }
    std::vector<uint32_t> sym;
    for (uint64_t ci = 0; ci < c.chunks.size(); ++ci) {
        const uint64_t r0 = ci << c.log2_rows, r1 = std::min<uint64_t>(d.num_rows, (ci + 1) << c.log2_rows);
        const uint64_t s0 = d.offsets[r0], s1 = d.offsets[r1];
        sym.assign(d.cols + s0, d.cols + s1);
        for (uint64_t r = r0; r < r1; ++r) {  // rows are sets: sort, reject repeats and bad ids
            uint32_t *b = sym.data() + (d.offsets[r] - s0), *e = sym.data() + (d.offsets[r + 1] - s0);
            std::sort(b, e);
            for (uint32_t *p = b; p != e; ++p) {
                if (*p >= d.num_columns) {
                    set_error("column id >= num_columns");
                    return MBRWT_ERR_INVALID;
                }
                if (p != b && p[-1] == *p) {
                    set_error("row lists a column twice");
                    return MBRWT_ERR_INVALID;
                }
            }
        }
        WtChunkDev &ch = c.chunks[ci];
        ch.str0 = s0;
        const uint64_t len = s1 - s0;
        if ((rc = ensure(c.ws_a, std::max<uint64_t>(len, 1) * sizeof(uint32_t)))) return rc;
        if ((rc = ensure(c.ws_b, std::max<uint64_t>(len, 1) * sizeof(uint32_t)))) return rc;
        if (len)
            MBRWT_HIP(hipMemcpyAsync(c.ws_a.buf, sym.data(), len * sizeof(uint32_t), hipMemcpyHostToDevice, c.stream));
        if ((rc = build_chunk(c, ch, reinterpret_cast<uint32_t *>(c.ws_a.buf), reinterpret_cast<uint32_t *>(c.ws_b.buf),
                              len, c.stream)))
            return rc;
    }
    return finish(c);
}

int build_synthetic_wt(WtCtx &c, const mbrwt_binrel_synth_desc &d) {
    if (!(d.density >= 0.0 && d.density <= 1.0) || d.num_columns == 0 || d.num_columns > 0xFFFFFFFFull) {
        set_error("invalid synthetic BinRel description");
        return MBRWT_ERR_INVALID;
    }
    int rc = init_common(c, c.device, d.num_rows, d.num_columns);
    if (rc) return rc;
    const uint64_t T = d.density <= 0 ? 0 : d.density >= 1 ? ~0ull : (uint64_t)(d.density * 18446744073709551616.0);
    const uint64_t R = 1ull << c.log2_rows;
    if ((rc = ensure(c.ws_io, (R + 1) * 2 * sizeof(uint32_t)))) return rc;
    uint32_t *d_cnt = reinterpret_cast<uint32_t *>(c.ws_io.buf);
    uint32_t *d_off = d_cnt + R + 1;
    size_t scan_bytes = 0;
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, d_cnt, d_off, (int)(R + 1), c.stream));
    uint64_t str0 = 0;
    for (uint64_t ci = 0; ci < c.chunks.size(); ++ci) {
        const uint64_t r0 = ci << c.log2_rows, nr = std::min<uint64_t>(d.num_rows - r0, R);
        hipLaunchKernelGGL(k_wt_synth_count, dim3(grid_for(nr)), dim3(256), 0, c.stream, r0, nr,
                           (uint32_t)d.num_columns, T, d.seed, d_cnt);
        MBRWT_HIP(hipMemsetAsync(d_cnt + nr, 0, sizeof(uint32_t), c.stream));
        if ((rc = ensure(c.ws_scan, scan_bytes + 16))) return rc;
        MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(c.ws_scan.buf, scan_bytes, d_cnt, d_off, (int)(nr + 1), c.stream));
        MBRWT_HIP(hipMemcpyAsync(c.h_scalars, d_off + nr, sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
        MBRWT_HIP(hipStreamSynchronize(c.stream));
        uint32_t len32 = 0;
        std::memcpy(&len32, c.h_scalars, sizeof(uint32_t));
        const uint64_t len = len32;
        if ((rc = ensure(c.ws_a, std::max<uint64_t>(len, 1) * sizeof(uint32_t)))) return rc;
        if ((rc = ensure(c.ws_b, std::max<uint64_t>(len, 1) * sizeof(uint32_t)))) return rc;
        hipLaunchKernelGGL(k_wt_synth_write, dim3(grid_for(nr)), dim3(256), 0, c.stream, r0, nr,
                           (uint32_t)d.num_columns, T, d.seed, d_off, str0, reinterpret_cast<uint32_t *>(c.ws_a.buf),
                           c.d_offsets);
        MBRWT_HIP(hipGetLastError());
        WtChunkDev &ch = c.chunks[ci];
        ch.str0 = str0;
        if ((rc = build_chunk(c, ch, reinterpret_cast<uint32_t *>(c.ws_a.buf), reinterpret_cast<uint32_t *>(c.ws_b.buf),
                              len, c.stream)))
            return rc;
        str0 += len;
    }
    c.num_relations = str0;
    MBRWT_HIP(hipMemcpyAsync(c.d_offsets + d.num_rows, &c.num_relations, sizeof(uint64_t), hipMemcpyHostToDevice,
                             c.stream));
    MBRWT_HIP(hipStreamSynchronize(c.stream));
    // the build workspaces are not needed by the queries
    for (Workspace *ws : {&c.ws_a, &c.ws_b, &c.ws_c}) {
        if (ws->buf) MBRWT_HIP(hipFree(ws->buf));
        ws->buf = nullptr;
        ws->bytes = 0;
    }
    return finish(c);
}

int wt_get_rows(WtCtx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_csr, uint32_t *d_cols, uint64_t cap,
                uint64_t *needed, hipStream_t s) {
    const WtParams P = c.params();
    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 4 * sizeof(uint64_t), s));
    MBRWT_HIP(hipMemsetAsync(d_csr, 0, sizeof(uint64_t), s));
    if (!n) {
        if (needed) *needed = 0;
        return MBRWT_OK;
    }
    hipLaunchKernelGGL(k_wt_lengths, dim3(grid_for(n)), dim3(256), 0, s, P, d_rows, n, d_csr + 1);
    MBRWT_HIP(hipGetLastError());
    size_t scan_bytes = 0;
    MBRWT_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes, d_csr + 1, d_csr + 1, (int)n, s));
    int rc;
    if ((rc = ensure(c.ws_scan, scan_bytes + 16))) return rc;
    MBRWT_HIP(hipcub::DeviceScan::InclusiveSum(c.ws_scan.buf, scan_bytes, d_csr + 1, d_csr + 1, (int)n, s));
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, d_csr + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars + 1, c.d_scalars + 2, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (c.h_scalars[1] & 1) {
        set_error("row out of range");
        return MBRWT_ERR_RANGE;
    }
    const uint64_t total = c.h_scalars[0];
    if (needed) *needed = total;
    if (total > cap || (total && !d_cols)) {
        set_error("label buffer too small (see cols_needed)");
        return MBRWT_ERR_CAPACITY;
    }
    if (!total) return MBRWT_OK;
    if (c.timing) MBRWT_HIP(hipEventRecord(c.ev0, s));
    const uint64_t tiles = (n + kWtTile - 1) / kWtTile;
    hipLaunchKernelGGL(k_wt_decode, dim3((unsigned)std::min<uint64_t>(tiles, 1u << 20)), dim3(kWtTile), 0, s, P,
                       d_rows, n, d_csr, d_cols);
    MBRWT_HIP(hipGetLastError());
    if (c.timing) {
        MBRWT_HIP(hipEventRecord(c.ev1, s));
        MBRWT_HIP(hipEventSynchronize(c.ev1));
        float ms = 0;
        MBRWT_HIP(hipEventElapsedTime(&ms, c.ev0, c.ev1));
        c.timing_ms += ms;
        c.timing_launches += 1;
    }
    return MBRWT_OK;
}

int wt_get_batch(WtCtx &c, const uint64_t *d_rows, const uint64_t *d_cols, uint64_t n, uint8_t *d_out, hipStream_t s) {
    if (!n) return MBRWT_OK;
    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 4 * sizeof(uint64_t), s));
    hipLaunchKernelGGL(k_wt_get, dim3(grid_for(n)), dim3(256), 0, s, c.params(), d_rows, d_cols, n, d_out);
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars + 2, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (c.h_scalars[0] & 1) {
        set_error("row or column out of range");
        return MBRWT_ERR_RANGE;
    }
    return MBRWT_OK;
}

int wt_get_column(WtCtx &c, uint64_t column, uint64_t *d_rows, uint64_t cap, uint64_t *needed, hipStream_t s) {
    if (column >= c.num_columns) {
        set_error("column out of range");
        return MBRWT_ERR_RANGE;
    }
    const uint64_t nch = c.chunks.size();
    if (!nch) {
        if (needed) *needed = 0;
        return MBRWT_OK;
    }
    int rc;
    if ((rc = ensure(c.ws_io, nch * (sizeof(uint32_t) + 2 * sizeof(uint64_t)) + 64))) return rc;
    uint64_t *d_cnt = reinterpret_cast<uint64_t *>(c.ws_io.buf);
    uint64_t *d_coff = d_cnt + nch;
    uint32_t *d_start = reinterpret_cast<uint32_t *>(d_coff + nch);
    const WtParams P = c.params();
    hipLaunchKernelGGL(k_wt_col_range, dim3(grid_for(nch)), dim3(256), 0, s, P, nch, (uint32_t)column, d_start, d_cnt);
    MBRWT_HIP(hipGetLastError());
    size_t scan_bytes = 0;
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, d_cnt, d_coff, (int)nch, s));
    if ((rc = ensure(c.ws_scan, scan_bytes + 16))) return rc;
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(c.ws_scan.buf, scan_bytes, d_cnt, d_coff, (int)nch, s));
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, d_coff + nch - 1, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars + 1, d_cnt + nch - 1, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    const uint64_t total = c.h_scalars[0] + c.h_scalars[1];
    if (needed) *needed = total;
    if (total > cap || (total && !d_rows)) {
        set_error("row buffer too small (see rows_needed)");
        return MBRWT_ERR_CAPACITY;
    }
    if (!total) return MBRWT_OK;
    hipLaunchKernelGGL(k_wt_col_lift, dim3(grid_for(total)), dim3(256), 0, s, P, nch, (uint32_t)column, d_start,
                       d_coff, total, d_rows);
    MBRWT_HIP(hipGetLastError());
    return MBRWT_OK;
}

// classify over BinRel-WT rows (classify.hip's driver with wt_get_rows)
ClassifyIo wt_io(WtCtx &c) { return ClassifyIo{&c.ws_cls_off, &c.ws_cls_cols, &c.ws_cls_cnt, &c.ws_scan}; }
ClassifyRowsFn wt_rows(WtCtx &c, const uint64_t *d_rows, uint64_t n_rows, hipStream_t s) {
    return [&c, d_rows, n_rows, s](uint64_t *d_off, uint32_t *d_cols, uint64_t cap, uint64_t *need) {
        return wt_get_rows(c, d_rows, n_rows, d_off, d_cols, cap, need, s);
    };
}

WtCtx *W(mbrwt_wt *p) { return reinterpret_cast<WtCtx *>(p); }
const WtCtx *W(const mbrwt_wt *p) { return reinterpret_cast<const WtCtx *>(p); }

template <class F>
int guarded(const char *what, F &&f) {
    try {
        return f();
    } catch (const std::bad_alloc &) {
        set_error(std::string("out of host memory in ") + what);
        return MBRWT_ERR_NOMEM;
    } catch (...) {
        set_error(std::string("unexpected exception in ") + what);
        return MBRWT_ERR_INVALID;
    }
}

}  // namespace
}  // namespace mbrwt

using mbrwt::W;
using mbrwt::WtCtx;

extern "C" {

int mbrwt_wt_create(const mbrwt_binrel_desc *desc, int device, mbrwt_wt **out) {
    if (!desc || !out) {
        mbrwt::set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    *out = nullptr;
    return mbrwt::guarded("mbrwt_wt_create", [&] {
        std::unique_ptr<WtCtx> c(new WtCtx());
        c->device = device;
        int rc = mbrwt::build_from_csr(*c, *desc);
        if (rc) return rc;
        *out = reinterpret_cast<mbrwt_wt *>(c.release());
        return (int)MBRWT_OK;
    });
}

int mbrwt_wt_create_synthetic(const mbrwt_binrel_synth_desc *desc, int device, mbrwt_wt **out) {
    if (!desc || !out) {
        mbrwt::set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    *out = nullptr;
    return mbrwt::guarded("mbrwt_wt_create_synthetic", [&] {
        std::unique_ptr<WtCtx> c(new WtCtx());
        c->device = device;
        int rc = mbrwt::build_synthetic_wt(*c, *desc);
        if (rc) return rc;
        *out = reinterpret_cast<mbrwt_wt *>(c.release());
        return (int)MBRWT_OK;
    });
}

void mbrwt_wt_destroy(mbrwt_wt *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(W(ctx)->device);
    delete W(ctx);
}

uint64_t mbrwt_wt_num_rows(const mbrwt_wt *ctx) { return ctx ? W(ctx)->num_rows : 0; }
uint64_t mbrwt_wt_num_columns(const mbrwt_wt *ctx) { return ctx ? W(ctx)->num_columns : 0; }
uint64_t mbrwt_wt_num_relations(const mbrwt_wt *ctx) { return ctx ? W(ctx)->num_relations : 0; }
uint64_t mbrwt_wt_device_bytes(const mbrwt_wt *ctx) { return ctx ? W(ctx)->device_bytes : 0; }

int mbrwt_wt_get_rows_device(mbrwt_wt *ctx, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets,
                             uint32_t *d_cols, uint64_t cols_cap, uint64_t *cols_needed, void *stream) {
    if (!ctx || !d_offsets || (n && !d_rows)) {
        mbrwt::set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    WtCtx &c = *W(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    mbrwt::WsFence fence_(c.fence, reinterpret_cast<hipStream_t>(stream));
    return mbrwt::guarded("mbrwt_wt_get_rows_device", [&] {
        MBRWT_HIP(hipSetDevice(c.device));
        return mbrwt::wt_get_rows(c, d_rows, n, d_offsets, d_cols, d_cols ? cols_cap : 0, cols_needed,
                                  reinterpret_cast<hipStream_t>(stream));
    });
}

int mbrwt_wt_get_rows(mbrwt_wt *ctx, const uint64_t *rows, uint64_t n, uint64_t *offsets, uint32_t *cols,
                      uint64_t cols_cap, uint64_t *cols_needed) {
    if (!ctx || !offsets || (n && !rows)) {
        mbrwt::set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    WtCtx &c = *W(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    mbrwt::WsFence fence_(c.fence, c.stream);
    return mbrwt::guarded("mbrwt_wt_get_rows", [&] {
        MBRWT_HIP(hipSetDevice(c.device));
        int rc;
        if ((rc = mbrwt::ensure(c.ws_a, (2 * n + 1) * sizeof(uint64_t)))) return rc;
        if ((rc = mbrwt::ensure(c.ws_b, std::max<uint64_t>(cols_cap, 1) * sizeof(uint32_t)))) return rc;
        uint64_t *d_rows = reinterpret_cast<uint64_t *>(c.ws_a.buf);
        uint64_t *d_off = d_rows + n;
        if (n) MBRWT_HIP(hipMemcpyAsync(d_rows, rows, n * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream));
        uint64_t need = 0;
        rc = mbrwt::wt_get_rows(c, d_rows, n, d_off, cols ? reinterpret_cast<uint32_t *>(c.ws_b.buf) : nullptr,
                                cols ? cols_cap : 0, &need, c.stream);
        if (cols_needed) *cols_needed = need;
        if (rc) return rc;
        MBRWT_HIP(hipMemcpyAsync(offsets, d_off, (n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
        if (need) MBRWT_HIP(hipMemcpyAsync(cols, c.ws_b.buf, need * sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
        MBRWT_HIP(hipStreamSynchronize(c.stream));
        return (int)MBRWT_OK;
    });
}

int mbrwt_wt_get_batch_device(mbrwt_wt *ctx, const uint64_t *d_rows, const uint64_t *d_cols, uint64_t n,
                              uint8_t *d_out, void *stream) {
    if (!ctx || (n && (!d_rows || !d_cols || !d_out))) {
        mbrwt::set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    WtCtx &c = *W(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    mbrwt::WsFence fence_(c.fence, reinterpret_cast<hipStream_t>(stream));
    return mbrwt::guarded("mbrwt_wt_get_batch_device", [&] {
        MBRWT_HIP(hipSetDevice(c.device));
        return mbrwt::wt_get_batch(c, d_rows, d_cols, n, d_out, reinterpret_cast<hipStream_t>(stream));
    });
}

int mbrwt_wt_get_batch(mbrwt_wt *ctx, const uint64_t *rows, const uint64_t *cols, uint64_t n, uint8_t *out) {
    if (!ctx || (n && (!rows || !cols || !out))) {
        mbrwt::set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    WtCtx &c = *W(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    mbrwt::WsFence fence_(c.fence, c.stream);
    return mbrwt::guarded("mbrwt_wt_get_batch", [&] {
        MBRWT_HIP(hipSetDevice(c.device));
        if (!n) return (int)MBRWT_OK;
        int rc;
        if ((rc = mbrwt::ensure(c.ws_a, n * (2 * sizeof(uint64_t) + 1)))) return rc;
        uint64_t *d_r = reinterpret_cast<uint64_t *>(c.ws_a.buf);
        uint64_t *d_c = d_r + n;
        uint8_t *d_o = reinterpret_cast<uint8_t *>(d_c + n);
        MBRWT_HIP(hipMemcpyAsync(d_r, rows, n * 8, hipMemcpyHostToDevice, c.stream));
        MBRWT_HIP(hipMemcpyAsync(d_c, cols, n * 8, hipMemcpyHostToDevice, c.stream));
        rc = mbrwt::wt_get_batch(c, d_r, d_c, n, d_o, c.stream);
        if (rc) return rc;
        MBRWT_HIP(hipMemcpyAsync(out, d_o, n, hipMemcpyDeviceToHost, c.stream));
        MBRWT_HIP(hipStreamSynchronize(c.stream));
        return (int)MBRWT_OK;
    });
}

int mbrwt_wt_get_column_device(mbrwt_wt *ctx, uint64_t column, uint64_t *d_rows, uint64_t rows_cap,
                               uint64_t *rows_needed, void *stream) {
    if (!ctx) {
        mbrwt::set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    WtCtx &c = *W(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    mbrwt::WsFence fence_(c.fence, reinterpret_cast<hipStream_t>(stream));
    return mbrwt::guarded("mbrwt_wt_get_column_device", [&] {
        MBRWT_HIP(hipSetDevice(c.device));
        return mbrwt::wt_get_column(c, column, d_rows, d_rows ? rows_cap : 0, rows_needed,
                                    reinterpret_cast<hipStream_t>(stream));
    });
}

int mbrwt_wt_get_column(mbrwt_wt *ctx, uint64_t column, uint64_t *rows, uint64_t rows_cap, uint64_t *rows_needed) {
    if (!ctx) {
        mbrwt::set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    WtCtx &c = *W(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    mbrwt::WsFence fence_(c.fence, c.stream);
    return mbrwt::guarded("mbrwt_wt_get_column", [&] {
        MBRWT_HIP(hipSetDevice(c.device));
        int rc;
        if ((rc = mbrwt::ensure(c.ws_b, std::max<uint64_t>(rows_cap, 1) * sizeof(uint64_t)))) return rc;
        uint64_t need = 0;
        rc = mbrwt::wt_get_column(c, column, reinterpret_cast<uint64_t *>(c.ws_b.buf), rows ? rows_cap : 0, &need,
                                  c.stream);
        if (rows_needed) *rows_needed = need;
        if (rc) return rc;
        if (need) MBRWT_HIP(hipMemcpyAsync(rows, c.ws_b.buf, need * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
        MBRWT_HIP(hipStreamSynchronize(c.stream));
        return (int)MBRWT_OK;
    });
}

int mbrwt_wt_set_option(mbrwt_wt *ctx, int option, int64_t value) {
    if (!ctx) return MBRWT_ERR_INVALID;
    WtCtx &c = *W(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    if (option == MBRWT_OPT_TIMING) {
        c.timing = value != 0;
        return MBRWT_OK;
    }
    mbrwt::set_error("unknown option");
    return MBRWT_ERR_INVALID;
}

int mbrwt_wt_take_timing(mbrwt_wt *ctx, double *kernel_ms, uint64_t *launches) {
    if (!ctx) return MBRWT_ERR_INVALID;
    WtCtx &c = *W(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    if (kernel_ms) *kernel_ms = c.timing_ms;
    if (launches) *launches = c.timing_launches;
    c.timing_ms = 0;
    c.timing_launches = 0;
    return MBRWT_OK;
}


int mbrwt_wt_get_labels_batch_device(mbrwt_wt *ctx, const uint64_t *d_rows, uint64_t n_rows,
                                     const uint64_t *d_read_offsets, uint64_t n_reads, double presence_ratio,
                                     uint64_t *d_label_offsets, uint32_t *d_labels, uint64_t labels_cap,
                                     uint64_t *labels_needed, void *stream) {
    if (!ctx || (n_rows && !d_rows) || !d_read_offsets || !d_label_offsets) {
        mbrwt::set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    WtCtx &c = *W(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    mbrwt::WsFence fence_(c.fence, reinterpret_cast<hipStream_t>(stream));
    return mbrwt::guarded("mbrwt_wt_get_labels_batch_device", [&] {
        MBRWT_HIP(hipSetDevice(c.device));
        const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
        return mbrwt::classify_labels(mbrwt::wt_io(c), mbrwt::wt_rows(c, d_rows, n_rows, s), c.num_columns, n_rows,
                                      d_read_offsets, n_reads, presence_ratio, d_label_offsets, d_labels,
                                      d_labels ? labels_cap : 0, labels_needed, s);
    });
}

int mbrwt_wt_get_top_labels_batch_device(mbrwt_wt *ctx, const uint64_t *d_rows, uint64_t n_rows,
                                         const uint64_t *d_read_offsets, uint64_t n_reads, uint64_t num_top,
                                         uint64_t *d_label_offsets, uint32_t *d_labels, uint64_t *d_counts,
                                         uint64_t labels_cap, uint64_t *labels_needed, void *stream) {
    if (!ctx || (n_rows && !d_rows) || !d_read_offsets || !d_label_offsets) {
        mbrwt::set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    WtCtx &c = *W(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    mbrwt::WsFence fence_(c.fence, reinterpret_cast<hipStream_t>(stream));
    return mbrwt::guarded("mbrwt_wt_get_top_labels_batch_device", [&] {
        MBRWT_HIP(hipSetDevice(c.device));
        const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
        const bool out = d_labels && d_counts;
        return mbrwt::classify_top_labels(mbrwt::wt_io(c), mbrwt::wt_rows(c, d_rows, n_rows, s), c.num_columns,
                                          n_rows, d_read_offsets, n_reads, num_top, d_label_offsets, d_labels,
                                          d_counts, out ? labels_cap : 0, labels_needed, s);
    });
}

// host-buffer forms: rows | read offsets | label offsets in ws_a, labels (+ counts) in ws_b
int mbrwt_wt_get_labels_batch(mbrwt_wt *ctx, const uint64_t *rows, uint64_t n_rows, const uint64_t *read_offsets,
                              uint64_t n_reads, double presence_ratio, uint64_t *label_offsets, uint32_t *labels,
                              uint64_t labels_cap, uint64_t *labels_needed) {
    if (!ctx || (n_rows && !rows) || !read_offsets || !label_offsets) {
        mbrwt::set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    WtCtx &c = *W(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    mbrwt::WsFence fence_(c.fence, c.stream);
    return mbrwt::guarded("mbrwt_wt_get_labels_batch", [&] {
        MBRWT_HIP(hipSetDevice(c.device));
        int rc;
        if ((rc = mbrwt::ensure(c.ws_a, (n_rows + 2 * (n_reads + 1)) * sizeof(uint64_t)))) return rc;
        if ((rc = mbrwt::ensure(c.ws_b, std::max<uint64_t>(labels_cap, 1) * sizeof(uint32_t)))) return rc;
        uint64_t *d_rows = reinterpret_cast<uint64_t *>(c.ws_a.buf);
        uint64_t *d_roff = d_rows + n_rows, *d_loff = d_roff + n_reads + 1;
        if (n_rows) MBRWT_HIP(hipMemcpyAsync(d_rows, rows, n_rows * 8, hipMemcpyHostToDevice, c.stream));
        MBRWT_HIP(hipMemcpyAsync(d_roff, read_offsets, (n_reads + 1) * 8, hipMemcpyHostToDevice, c.stream));
        uint64_t need = 0;
        rc = mbrwt::classify_labels(mbrwt::wt_io(c), mbrwt::wt_rows(c, d_rows, n_rows, c.stream), c.num_columns,
                                    n_rows, d_roff, n_reads, presence_ratio, d_loff,
                                    labels ? reinterpret_cast<uint32_t *>(c.ws_b.buf) : nullptr,
                                    labels ? labels_cap : 0, &need, c.stream);
        if (labels_needed) *labels_needed = need;
        if (rc) return rc;
        MBRWT_HIP(hipMemcpyAsync(label_offsets, d_loff, (n_reads + 1) * 8, hipMemcpyDeviceToHost, c.stream));
        if (need) MBRWT_HIP(hipMemcpyAsync(labels, c.ws_b.buf, need * 4, hipMemcpyDeviceToHost, c.stream));
        MBRWT_HIP(hipStreamSynchronize(c.stream));
        return (int)MBRWT_OK;
    });
}

int mbrwt_wt_get_top_labels_batch(mbrwt_wt *ctx, const uint64_t *rows, uint64_t n_rows, const uint64_t *read_offsets,
                                  uint64_t n_reads, uint64_t num_top, uint64_t *label_offsets, uint32_t *labels,
                                  uint64_t *counts, uint64_t labels_cap, uint64_t *labels_needed) {
    if (!ctx || (n_rows && !rows) || !read_offsets || !label_offsets) {
        mbrwt::set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    WtCtx &c = *W(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    mbrwt::WsFence fence_(c.fence, c.stream);
    return mbrwt::guarded("mbrwt_wt_get_top_labels_batch", [&] {
        MBRWT_HIP(hipSetDevice(c.device));
        int rc;
        if ((rc = mbrwt::ensure(c.ws_a, (n_rows + 2 * (n_reads + 1)) * sizeof(uint64_t)))) return rc;
        const uint64_t lab_words = (std::max<uint64_t>(labels_cap, 1) + 1) & ~1ull;
        if ((rc = mbrwt::ensure(c.ws_b, lab_words * 4 + std::max<uint64_t>(labels_cap, 1) * 8))) return rc;
        uint64_t *d_rows = reinterpret_cast<uint64_t *>(c.ws_a.buf);
        uint64_t *d_roff = d_rows + n_rows, *d_loff = d_roff + n_reads + 1;
        uint32_t *d_lab = reinterpret_cast<uint32_t *>(c.ws_b.buf);
        uint64_t *d_cnt = reinterpret_cast<uint64_t *>(d_lab + lab_words);
        if (n_rows) MBRWT_HIP(hipMemcpyAsync(d_rows, rows, n_rows * 8, hipMemcpyHostToDevice, c.stream));
        MBRWT_HIP(hipMemcpyAsync(d_roff, read_offsets, (n_reads + 1) * 8, hipMemcpyHostToDevice, c.stream));
        uint64_t need = 0;
        const bool out = labels && counts;
        rc = mbrwt::classify_top_labels(mbrwt::wt_io(c), mbrwt::wt_rows(c, d_rows, n_rows, c.stream), c.num_columns,
                                        n_rows, d_roff, n_reads, num_top, d_loff, out ? d_lab : nullptr,
                                        out ? d_cnt : nullptr, out ? labels_cap : 0, &need, c.stream);
        if (labels_needed) *labels_needed = need;
        if (rc) return rc;
        MBRWT_HIP(hipMemcpyAsync(label_offsets, d_loff, (n_reads + 1) * 8, hipMemcpyDeviceToHost, c.stream));
        if (need) {
            MBRWT_HIP(hipMemcpyAsync(labels, d_lab, need * 4, hipMemcpyDeviceToHost, c.stream));
            MBRWT_HIP(hipMemcpyAsync(counts, d_cnt, need * 8, hipMemcpyDeviceToHost, c.stream));
        }
        MBRWT_HIP(hipStreamSynchronize(c.stream));
        return (int)MBRWT_OK;
    });
}

}  // extern "C"

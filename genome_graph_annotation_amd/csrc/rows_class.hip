// rows_class.hip -- RECORD CLASSES: one copy of every distinct row record.
//
// A row's record (rows.hip) is a function of its label set alone: the masks
// of the descent BRWT::get_row takes (BRWT.cpp:26-53) are fixed by which
// columns are set.  Rows with the same label set therefore hold byte-equal
// records, and on correlated data most rows repeat one of few label sets --
// the reference's own `uniform_rows` / `weighted_rows` generators
// (experiments/main.cpp:232-285, data_generation.cpp:114-200), and the
// colour classes of real k-mer annotations.  BRWT has no mechanism for
// repeated ROWS (its index columns are stored per row), so
// there the row records cost 32 bytes a row however few distinct rows exist.
//
// The class form replaces the block image by
//   * a dictionary: the D distinct records as a block image of one record per
//     64-byte block (S = 1; records longer than a block in the spill area), and
//   * a class index: w = ceil(log2 D) bits per row, packed LSB-first in u32
//     words -- row r's class is bits [r w, r w + w).
// get_rows maps the batch's row ids through the index (one random read per
// row, k_class_map) and runs the unchanged traversal over the dictionary,
// whose blocks are small enough to stay in the L2 / MALL.
//
// Build (rows_classes_build, after the block image of every range is
// written): a 64-bit FNV-1a hash of every row's record, a radix sort of
// (hash, row), class ids as the running count of distinct hashes, and a
// byte-for-byte comparison of every row's record with its class
// representative's -- a hash collision keeps the block image, so the form is
// exact by construction.  Layout AUTO first hashes a strided sample of 2^20
// rows and builds the classes only when at least a tenth of the sample
// repeats a record (a sample of one row in 100 of a matrix with 100 copies of
// each row already sees 38 % repeats; i.i.d. columns see almost none), then
// keeps them when there are at most half as many classes as rows and they
// at least halve the image.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>

#include "mbrwt_internal.hpp"
#include "rows_record.hpp"

namespace mbrwt {
namespace {

constexpr uint64_t kFnvBasis = 0xcbf29ce484222325ull;
constexpr uint64_t kFnvPrime = 0x100000001b3ull;
constexpr uint32_t kClassB = 64;  // dictionary block bytes (one record per block)
constexpr uint64_t kSampleRows = 1ull << 20;

struct RecordRef {
    uint64_t masks;
    uint32_t count, len;
};

// row r's record: its first mask byte, label count and mask bytes (the walk
// over the RWT table reads exactly the record's bytes); false if the walk
// fails (a corrupt image)
__device__ bool record_of(const RowsView &v, const uint32_t *table, uint64_t r, RecordRef &rr) {
    rows_locate(v, r, rr.masks, rr.count);
    rr.len = 0;
    if (!rr.count) return true;
    uint32_t hi = 0;
    const uint64_t m = rr.masks;
    const bool ok = record_walk_bytes(
        v, table,
        [&](uint32_t o) {
            hi = o + 1 > hi ? o + 1 : hi;
            return (uint32_t)gld_at<uint8_t>(m + o);
        },
        rr.count, [](uint32_t) {}, [](uint32_t) {});
    rr.len = hi;
    return ok;
}

__device__ uint64_t record_hash(const RecordRef &rr) {
    uint64_t h = kFnvBasis;
    for (uint32_t k = 0; k < 4; ++k) h = (h ^ ((rr.count >> (8 * k)) & 0xFFu)) * kFnvPrime;
    for (uint32_t o = 0; o < rr.len; ++o) h = (h ^ gld_at<uint8_t>(rr.masks + o)) * kFnvPrime;
    return h;
}

// the records of rows row0 + i * stride (i < items): hash -> keys[i], the row -> vals[i]
__global__ __launch_bounds__(256) void k_class_hash(RowsView v, const uint32_t *table, uint64_t row0, uint64_t stride,
                                                    uint64_t items, uint64_t *keys, uint64_t *vals,
                                                    unsigned long long *err) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < items; i += gs) {
        const uint64_t r = row0 + i * stride;
        RecordRef rr;
        if (!record_of(v, table, r, rr)) atomicOr(err, 1ull);
        gst(keys + i, record_hash(rr));
        if (vals) gst(vals + i, r);
    }
}

// 1 where a sorted key starts a run of equal keys
struct HeadFlag {
    const uint64_t *keys;
    __host__ __device__ uint64_t operator()(const uint64_t &i) const { return (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u; }
};

// rep[class] = the first row of every run (cid1: the 1-based class of each sorted position)
__global__ __launch_bounds__(256) void k_class_reps(const uint64_t *keys, const uint64_t *rows, const uint64_t *cid1,
                                                    uint64_t n, uint64_t *rep) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs)
        if (i == 0 || gld(keys + i) != gld(keys + i - 1)) gst(rep + gld(cid1 + i) - 1, gld(rows + i));
}

// every row: its record equals its class representative's (else err bit 1:
// a hash collision), and its class into the packed index (fields may share
// words: atomic ors into a zeroed index)
__global__ __launch_bounds__(256) void k_class_assign(RowsView v, const uint32_t *table, const uint64_t *rows,
                                                      const uint64_t *cid1, const uint64_t *rep, uint64_t n,
                                                      uint32_t w, uint32_t *index, unsigned long long *err) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const uint64_t r = gld(rows + i), c = gld(cid1 + i) - 1, q = gld(rep + c);
        if (r != q) {
            RecordRef a, b;
            bool same = record_of(v, table, r, a) && record_of(v, table, q, b) && a.count == b.count && a.len == b.len;
            for (uint32_t o = 0; same && o < a.len; ++o)
                same = gld_at<uint8_t>(a.masks + o) == gld_at<uint8_t>(b.masks + o);
            if (!same) atomicOr(err, 2ull);
        }
        const uint64_t bit = r * w;
        const uint32_t sh = (uint32_t)(bit & 31);
        atomicOr(index + (bit >> 5), (uint32_t)(c << sh));
        if (sh + w > 32) atomicOr(index + (bit >> 5) + 1, (uint32_t)(c >> (32 - sh)));
    }
}

__device__ __forceinline__ bool class_spills(const RecordRef &rr) { return rr.count >= 255 || 2 + rr.len > kClassB; }
__device__ __forceinline__ uint32_t class_spill_units(const RecordRef &rr) { return (8 + rr.len + 15) / 16; }

// the dictionary's spill: [0] units, [1] spilled classes, [2] longer than a block
__global__ __launch_bounds__(256) void k_class_measure(RowsView v, const uint32_t *table, const uint64_t *rep,
                                                       uint64_t D, unsigned long long *acc) {
    unsigned long long units = 0, sp = 0, lng = 0;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < D; k += gs) {
        RecordRef rr;
        (void)record_of(v, table, gld(rep + k), rr);
        if (class_spills(rr)) {
            units += class_spill_units(rr);
            ++sp;
            lng += 8 + rr.len > kClassB ? 1u : 0u;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        units += __shfl_down(units, off);
        sp += __shfl_down(sp, off);
        lng += __shfl_down(lng, off);
    }
    if ((threadIdx.x & 63) == 0) {
        if (units) atomicAdd(acc + 0, units);
        if (sp) atomicAdd(acc + 1, sp);
        if (lng) atomicAdd(acc + 2, lng);
    }
}

// one thread per class: its block (entry byte, then the record inline or a
// spill entry) -- the block layout of rows.hip with S = 1
__global__ __launch_bounds__(256) void k_class_write(RowsView v, const uint32_t *table, const uint64_t *rep, uint64_t D,
                                                     uint8_t *blocks, uint8_t *spill, unsigned long long *spill_used) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < D; k += gs) {
        RecordRef rr;
        (void)record_of(v, table, gld(rep + k), rr);
        uint8_t *blk = blocks + k * kClassB;
        if (class_spills(rr)) {
            const uint64_t idx = atomicAdd(spill_used, (unsigned long long)class_spill_units(rr));
            uint8_t *se = spill + idx * 16;
            *reinterpret_cast<uint32_t *>(se) = rr.count;
            *reinterpret_cast<uint32_t *>(se + 4) = rr.len;
            for (uint32_t o = 0; o < rr.len; ++o) se[8 + o] = gld_at<uint8_t>(rr.masks + o);
            blk[0] = 1u | 0x80u;
            blk[1] = (uint8_t)std::min<uint32_t>(rr.count, 255);
            for (uint32_t b = 0; b < 4; ++b) blk[2 + b] = (uint8_t)(idx >> (8 * b));
        } else {
            blk[0] = 1u;
            blk[1] = (uint8_t)rr.count;
            for (uint32_t o = 0; o < rr.len; ++o) blk[2 + o] = gld_at<uint8_t>(rr.masks + o);
        }
    }
}

// the batch's row ids -> their classes (rows out of range -> D, which the
// dictionary kernels report as out of range)
__global__ __launch_bounds__(256) void k_class_map(const uint64_t *rows, uint64_t n, uint64_t num_rows,
                                                   const uint32_t *index, uint32_t w, uint64_t D, uint64_t *out) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const uint64_t r = gld(rows + i);
        gst(out + i, r < num_rows ? class_field(index, w, r) : D);
    }
}

// get_column: which classes hold the column (one byte per class)
__global__ __launch_bounds__(256) void k_class_has(RowsView v, const uint32_t *table, uint64_t D, uint32_t col,
                                                   uint8_t *has) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < D; k += gs) {
        uint64_t masks;
        uint32_t count;
        rows_locate(v, k, masks, count);
        bool hit = false;
        if (count) (void)record_walk(v, table, masks, count, [&](uint32_t c) { hit |= c == col; }, [](uint32_t) {});
        gst(has + k, (uint8_t)(hit ? 1 : 0));
    }
}
struct ClassHas {
    const uint32_t *index;
    uint32_t w;
    const uint8_t *has;
    __device__ bool operator()(const uint64_t &row) const { return has[class_field(index, w, row)] != 0; }
};
struct ClassHasCount {
    ClassHas f;
    __device__ uint64_t operator()(const uint64_t &row) const { return f(row) ? 1u : 0u; }
};

uint64_t grid_of(uint64_t items) { return std::max<uint64_t>(1, std::min<uint64_t>((items + 255) / 256, 65536)); }

// the table the record walks read: RWT, or TT for terminal records (r06)
const uint32_t *class_table(const RowsImage &im) { return im.term ? im.d_table3 : im.d_table; }
RowsView block_view(const RowsImage &im, uint64_t records) {
    RowsView v;
    v.blocks = (uint64_t)(uintptr_t)im.blocks;
    v.spill = (uint64_t)(uintptr_t)im.spill;
    v.magic = im.magic;
    v.num_rows = records;
    v.B = im.B;
    v.S = im.S;
    v.nib = im.nib ? 1u : 0u;
    v.term = im.term ? 1u : 0u;
    return v;
}

// device scratch of one build step, freed on every path out
struct Scratch {
    std::vector<void *> p;
    ~Scratch() {
        for (void *x : p) (void)hipFree(x);
    }
    // null when the device has no room -- a tolerated failure (the caller
    // keeps the block image), so HIP's sticky last error is cleared: the
    // next MBRWT_HIP(hipGetLastError()) of the same create call must not
    // fail the whole build with it
    template <class T>
    T *get(uint64_t count) {
        void *x = nullptr;
        if (hipMalloc(&x, std::max<uint64_t>(1, count) * sizeof(T)) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        p.push_back(x);
        return static_cast<T *>(x);
    }
};

}  // namespace

int rows_classes_build(RowsImage &im, uint64_t n, int mode, uint64_t *sample_distinct, hipStream_t s) {
    // (nibble-coded records: no classes -- a compact image of rows that do not
    // repeat; the two compressions answer different data)
    if (mode == 0 || im.var || im.nib || !im.blocks || !im.d_table || n < 2 || n > (1ull << 32)) return MBRWT_OK;
    const RowsView v = block_view(im, n);
    Scratch sc;
    unsigned long long *d_err = sc.get<unsigned long long>(4);
    if (!d_err) return MBRWT_OK;  // (no room: keep the block image)
    MBRWT_HIP(hipMemsetAsync(d_err, 0, 4 * sizeof(unsigned long long), s));
    unsigned long long h_err[4] = {0, 0, 0, 0};

    // AUTO: a strided sample first -- (almost) every record distinct (i.i.d.
    // columns, C2-C4): no classes, at the cost of hashing 2^20 records
    if (mode < 0 && n > kSampleRows) {
        const uint64_t m = kSampleRows, stride = n / m;
        uint64_t *k0 = sc.get<uint64_t>(m), *k1 = sc.get<uint64_t>(m), *d_cnt = sc.get<uint64_t>(1);
        if (!k0 || !k1 || !d_cnt) return MBRWT_OK;
        hipLaunchKernelGGL(k_class_hash, dim3((unsigned)grid_of(m)), dim3(256), 0, s, v, class_table(im), 0ull, stride, m,
                           k0, (uint64_t *)nullptr, d_err);
        MBRWT_HIP(hipGetLastError());
        size_t tb = 0, rb = 0;
        MBRWT_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, k0, k1, m, 0, 64, s));
        hipcub::CountingInputIterator<uint64_t> it(0);
        hipcub::TransformInputIterator<uint64_t, HeadFlag, hipcub::CountingInputIterator<uint64_t>> heads(it, HeadFlag{k1});
        MBRWT_HIP(hipcub::DeviceReduce::Sum(nullptr, rb, heads, d_cnt, m, s));
        void *tmp = sc.get<uint8_t>(std::max(tb, rb));
        if (!tmp) return MBRWT_OK;
        MBRWT_HIP(hipcub::DeviceRadixSort::SortKeys(tmp, tb, k0, k1, m, 0, 64, s));
        MBRWT_HIP(hipcub::DeviceReduce::Sum(tmp, rb, heads, d_cnt, m, s));
        uint64_t distinct = 0;
        MBRWT_HIP(hipMemcpyAsync(&distinct, d_cnt, 8, hipMemcpyDeviceToHost, s));
        MBRWT_HIP(hipMemcpyAsync(h_err, d_err, 8, hipMemcpyDeviceToHost, s));
        MBRWT_HIP(hipStreamSynchronize(s));
        if (sample_distinct) *sample_distinct = distinct;
        if (h_err[0]) return MBRWT_OK;
        if (distinct * 10 > m * 9) return MBRWT_OK;
    }

    // every row: (hash, row) sorted by hash -- four u64 arrays of n, the
    // sort's and the scan's temporary storage (hipcub's own figures), and the
    // class index at its widest (u32 per row); the build is skipped without
    // that much free memory, not failed
    size_t tb = 0, qb = 0;
    {
        hipcub::CountingInputIterator<uint64_t> it0(0);
        hipcub::TransformInputIterator<uint64_t, HeadFlag, hipcub::CountingInputIterator<uint64_t>> h0(
            it0, HeadFlag{nullptr});
        MBRWT_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (uint64_t *)nullptr, (uint64_t *)nullptr,
                                                     (uint64_t *)nullptr, (uint64_t *)nullptr, n, 0, 64, s));
        MBRWT_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, qb, h0, (uint64_t *)nullptr, n, s));
    }
    size_t free_b = 0, total_b = 0;
    MBRWT_HIP(hipMemGetInfo(&free_b, &total_b));
    const double need_b = 32.0 * (double)n + (double)std::max(tb, qb) + 4.0 * (double)n + (double)(256ull << 20);
    if (need_b > (double)free_b) return MBRWT_OK;
    uint64_t *keys_in = sc.get<uint64_t>(n), *vals_in = sc.get<uint64_t>(n);
    uint64_t *keys = sc.get<uint64_t>(n), *rows = sc.get<uint64_t>(n);
    if (!keys_in || !vals_in || !keys || !rows) return MBRWT_OK;
    hipLaunchKernelGGL(k_class_hash, dim3((unsigned)grid_of(n)), dim3(256), 0, s, v, class_table(im), 0ull, 1ull, n,
                       keys_in, vals_in, d_err);
    MBRWT_HIP(hipGetLastError());
    hipcub::CountingInputIterator<uint64_t> it(0);
    hipcub::TransformInputIterator<uint64_t, HeadFlag, hipcub::CountingInputIterator<uint64_t>> heads(it, HeadFlag{keys});
    void *tmp = sc.get<uint8_t>(std::max(tb, qb));
    if (!tmp) return MBRWT_OK;
    MBRWT_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys_in, keys, vals_in, rows, n, 0, 64, s));
    uint64_t *cid1 = keys_in;  // (free after the sort)
    uint64_t *rep = vals_in;
    MBRWT_HIP(hipcub::DeviceScan::InclusiveSum(tmp, qb, heads, cid1, n, s));
    uint64_t D = 0;
    MBRWT_HIP(hipMemcpyAsync(&D, cid1 + n - 1, 8, hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (!D) return MBRWT_OK;
    hipLaunchKernelGGL(k_class_reps, dim3((unsigned)grid_of(n)), dim3(256), 0, s, keys, rows, cid1, n, rep);
    MBRWT_HIP(hipGetLastError());
    uint32_t w = 1;
    while (w < 32 && (1ull << w) < D) ++w;
    const uint64_t index_words = (n * w + 31) / 32 + 2;  // (+2: class_field reads the next word)
    uint32_t *index = nullptr;
    if (hipMalloc(&index, index_words * 4) != hipSuccess) {
        (void)hipGetLastError();  // (tolerated: keep the block image)
        return MBRWT_OK;
    }
    MBRWT_HIP(hipMemsetAsync(index, 0, index_words * 4, s));
    hipLaunchKernelGGL(k_class_assign, dim3((unsigned)grid_of(n)), dim3(256), 0, s, v, class_table(im), rows, cid1, rep, n,
                       w, index, d_err);
    MBRWT_HIP(hipGetLastError());
    unsigned long long *d_acc = d_err + 1;  // [1] units, [2] spilled, [3] long
    hipLaunchKernelGGL(k_class_measure, dim3((unsigned)grid_of(D)), dim3(256), 0, s, v, class_table(im), rep, D, d_acc);
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipMemcpyAsync(h_err, d_err, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    const uint64_t spill_bytes = h_err[1] * 16;
    const uint64_t dict_bytes = D * kClassB + spill_bytes, new_bytes = dict_bytes + index_words * 4;
    // a collision or a corrupt record keeps the block image; AUTO keeps it too
    // unless rows repeat (at most half as many classes as rows -- not a mere
    // re-blocking of 128-byte blocks) and the classes at least halve it
    if (h_err[0] || (mode < 0 && (2 * D > n || 2 * new_bytes > im.bytes))) {
        (void)hipFree(index);
        return MBRWT_OK;
    }
    uint8_t *dblocks = nullptr, *dspill = nullptr;
    const uint64_t spill_cap = spill_bytes + kClassB + 256;
    if (hipMalloc(&dblocks, D * kClassB) != hipSuccess || hipMalloc(&dspill, spill_cap) != hipSuccess) {
        (void)hipGetLastError();  // (tolerated: keep the block image)
        if (dblocks) (void)hipFree(dblocks);
        (void)hipFree(index);
        return MBRWT_OK;
    }
    MBRWT_HIP(hipMemsetAsync(dblocks, 0, D * kClassB, s));
    MBRWT_HIP(hipMemsetAsync(dspill, 0, spill_cap, s));
    MBRWT_HIP(hipMemsetAsync(d_acc, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_class_write, dim3((unsigned)grid_of(D)), dim3(256), 0, s, v, class_table(im), rep, D, dblocks,
                       dspill, d_acc);
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipStreamSynchronize(s));
    // the dictionary replaces the block image
    (void)hipFree(im.blocks);
    (void)hipFree(im.spill);
    im.blocks = dblocks;
    im.spill = dspill;
    im.spill_cap = spill_cap;
    im.B = kClassB;
    im.S = 1;
    im.magic = 0;
    im.num_blocks = D;
    im.spill_bytes = spill_bytes;
    im.spilled_rows = h_err[2];
    im.long_rows = h_err[3];
    im.classes = index;
    im.class_bits = w;
    im.num_classes = D;
    im.class_index_bytes = index_words * 4;
    im.bytes = new_bytes;
    return MBRWT_OK;
}

int rows_class_map(Ctx &c, const uint64_t *d_rows, uint64_t n, const uint64_t **mapped, hipStream_t s) {
    const RowsImage &im = c.rows;
    if (int rc = ensure(c.ws_class, std::max<uint64_t>(1, n) * sizeof(uint64_t))) return rc;
    uint64_t *out = static_cast<uint64_t *>(c.ws_class.buf);
    if (n) {
        hipLaunchKernelGGL(k_class_map, dim3((unsigned)grid_of(n)), dim3(256), 0, s, d_rows, n, c.tree.num_rows,
                           im.classes, im.class_bits, im.num_classes, out);
        MBRWT_HIP(hipGetLastError());
    }
    *mapped = out;
    return MBRWT_OK;
}

int rows_class_get_column(Ctx &c, uint64_t column, uint64_t *d_rows, uint64_t rows_cap, uint64_t *rows_needed,
                          hipStream_t s) {
    const RowsImage &im = c.rows;
    const uint64_t n = c.tree.num_rows, D = im.num_classes;
    int rc;
    if ((rc = ensure(c.ws_class, D))) return rc;
    uint8_t *has = static_cast<uint8_t *>(c.ws_class.buf);
    hipLaunchKernelGGL(k_class_has, dim3((unsigned)grid_of(D)), dim3(256), 0, s, block_view(im, D), class_table(im), D,
                       (uint32_t)column, has);
    MBRWT_HIP(hipGetLastError());
    const ClassHas f{im.classes, im.class_bits, has};
    hipcub::CountingInputIterator<uint64_t> rows_it(0);
    hipcub::TransformInputIterator<uint64_t, ClassHasCount, hipcub::CountingInputIterator<uint64_t>> cnt_it(
        rows_it, ClassHasCount{f});
    size_t red_bytes = 0, sel_bytes = 0;
    uint64_t *d_num = reinterpret_cast<uint64_t *>(c.d_scalars);
    MBRWT_HIP(hipcub::DeviceReduce::Sum(nullptr, red_bytes, cnt_it, d_num, n, s));
    if ((rc = ensure(c.ws_scan, std::max<size_t>(red_bytes, 256)))) return rc;
    MBRWT_HIP(hipcub::DeviceReduce::Sum(c.ws_scan.buf, red_bytes, cnt_it, d_num, n, s));
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    const uint64_t need = c.h_scalars[0];
    if (rows_needed) *rows_needed = need;
    if (!d_rows || need > rows_cap) {
        if (need > rows_cap) {
            set_error("rows_cap too small");
            return MBRWT_ERR_CAPACITY;
        }
        return MBRWT_OK;
    }
    if (!need) return MBRWT_OK;
    MBRWT_HIP(hipcub::DeviceSelect::If(nullptr, sel_bytes, rows_it, d_rows, d_num, n, f, s));
    if ((rc = ensure(c.ws_scan, sel_bytes))) return rc;
    MBRWT_HIP(hipcub::DeviceSelect::If(c.ws_scan.buf, sel_bytes, rows_it, d_rows, d_num, n, f, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    return MBRWT_OK;
}

}  // namespace mbrwt

// rows_var.hip -- VARIABLE-LENGTH ROW RECORDS for dense rows (the RefSeq
// shape, BASELINE configs[2]).
//
// The block layout (rows.hip) gives each row ONE 64/128-byte block read; at
// 1 B x 3,173, d = 3.8 %, a row's pre-order record is ~160 bytes and would
// spill almost every row.  Here the records are contiguous in HBM, addressed
// by a directory, and a row costs one directory request plus the record's
// ~3 contiguous lines -- issued together, not as a chain of dependent reads.
//
// Record of a row (uniform trees: every leaf sits below a leaf parent with
// consecutive columns, K internal levels above them -- the basic
// partitioner's trees): the leaf parents ("units") the row reaches, as a
// bitmap over the units in DFS order, then the leaf mask of each reached
// unit, in unit order:
//     [u32 bitmap words x W][u8 mask per set bit][pad to 4 bytes]
// The upper levels' masks are implied (a node is reached iff a unit below
// it is), so the record holds exactly the leaf-level index bits of the
// row's descent plus one bit per unit -- at the RefSeq shape 156 bytes,
// against 160 for the pre-order masks.  For a uniform tree the units in DFS
// order are the leaf parents from left to right, so emitting every reached
// unit's labels in unit order IS BRWT::get_row's pre-order
// (BRWT.cpp:43-51).  A row without labels has no record (length 0).
//
// Directory: one 64-byte line per 13 rows: [u64 address of the line's first
// record][13 x u32 {offset from it in 4-byte units (17 bits) | label count
// << 17}][u32 offset of the end].  Ranges of a ranged build start at
// multiples of 360,360 = 13 x 27,720 rows, so lines never straddle ranges and
// each range's records are their own allocation.
//
// get_rows: k_var_locate (one thread per batch row: the directory entry ->
// record address, length, label count), one scan of the counts -> the CSR
// offsets, then k_var_decode: R = 64 / G rows per wave, G lanes per row; the
// tile's records are gathered into LDS by coalesced 16-byte loads (chunks of
// all rows numbered by a wave scan), each lane walks its share of the row's
// bitmap words emitting one label per lock-step iteration into the wave's
// LDS stage, and the tile's labels leave as 16-byte stores straight into the
// caller's CSR -- no temp region, no compaction.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>

#include "device_access.hpp"
#include "mbrwt_internal.hpp"
#include "rows_emit.hpp"

namespace mbrwt {

// ------------------------------------------------------------------------
// host tables
// ------------------------------------------------------------------------
bool var_prepare(const Tree &tree, RowsImage &im) {
    im.var_units.clear();
    im.var_unit_of.clear();
    im.var_anc.clear();
    const auto &N = tree.nodes;
    if (!im.uni || !im.mask1 || N.size() < 2) return false;
    const uint32_t rootd = tree.folded ? 0u : 1u;
    auto column_of = [&](const DevNode &d) { return tree.label_perm.empty() ? d.label : tree.label_perm[d.label]; };
    im.var_unit_of.assign(N.size(), 0xFFFFu);
    // DFS pre-order over the internal nodes; a leaf parent is a unit
    struct F {
        uint32_t v, c, depth;
    };
    std::vector<F> st{{rootd, 0, 0}};
    std::vector<uint32_t> path(im.uni + 1, 0);
    while (!st.empty()) {
        F &f = st.back();
        const DevNode &d = N[f.v];
        if (f.c == 0) path[std::min<uint32_t>(f.depth, im.uni)] = f.v;
        if (f.c == d.arity) {
            st.pop_back();
            continue;
        }
        const uint32_t w = d.first_child + f.c++;
        if (N[w].kind == KIND_LEAF) {
            if (f.c == 1) {  // f.v is a leaf parent (uniform: all its children are leaves)
                if (f.depth != im.uni || im.var_units.size() >= 0xFFFF) return false;
                im.var_unit_of[f.v] = (uint16_t)im.var_units.size();
                im.var_units.push_back(column_of(N[w]) | (uint32_t)d.arity << 16);
                for (uint32_t k = 0; k < im.uni; ++k) im.var_anc.push_back(path[k]);
            }
            continue;
        }
        st.push_back(F{w, 0, f.depth + 1});
    }
    im.var_W = ((uint32_t)im.var_units.size() + 31) / 32;
    // the basic partitioner's trees: unit u's first column is u * arity
    // (C3: 3,173 columns, 397 units of 8), so the decode computes it instead
    // of reading the unit table (one LDS read per label fewer)
    im.var_ustride = 0;
    if (im.var_units.size() >= 2) {
        const uint32_t a = (im.var_units[1] & 0xFFFFu) - (im.var_units[0] & 0xFFFFu);
        bool reg = a > 0 && (im.var_units[0] & 0xFFFFu) == 0;
        for (size_t u = 0; reg && u < im.var_units.size(); ++u)
            reg = (im.var_units[u] & 0xFFFFu) == u * a && (im.var_units[u] >> 16) <= a;
        if (reg) im.var_ustride = a;
    }
    return !im.var_units.empty();
}

namespace {

constexpr uint32_t kLineRows = 13;
constexpr uint32_t kOffBits = 17;  // 4-byte units from the line's base

// per row of a range: record length in 4-byte units and label count
__global__ __launch_bounds__(256) void k_var_measure(const DevNode *nodes, uint32_t folded, uint64_t n,
                                                     const uint16_t *__restrict__ unit_of, uint32_t W, uint16_t *units,
                                                     uint16_t *cnt, unsigned long long *acc) {
    unsigned long long lab = 0, bytes = 0, bad = 0;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gs) {
        uint32_t items = 0, labels = 0;
        const uint32_t L = emit_row_masks(nodes, folded != 0, (uint32_t)r, [&](uint32_t m, uint32_t, uint32_t d) {
            if (gld(unit_of + d) != 0xFFFFu) {
                ++items;
                labels += (uint32_t)__builtin_popcount(m);
            }
        });
        const uint32_t b = items ? 4 * W + items : 0;
        if (L == ~0u || L != labels || labels > 0x7FFFu) {
            ++bad;
            units[r] = 0;
            cnt[r] = 0;
            continue;
        }
        units[r] = (uint16_t)((b + 3) / 4);
        cnt[r] = (uint16_t)labels;
        lab += labels;
        bytes += (b + 3) / 4 * 4;
    }
    for (int off = 32; off > 0; off >>= 1) {
        lab += __shfl_down(lab, off);
        bytes += __shfl_down(bytes, off);
        bad += __shfl_down(bad, off);
    }
    if ((threadIdx.x & 63) == 0) {
        if (lab) atomicAdd(acc + 0, lab);
        if (bytes) atomicAdd(acc + 1, bytes);
        if (bad) atomicAdd(acc + 2, bad);
    }
}

// per row of a range: its record at chunk + 4 off[r] (the chunk is zeroed)
__global__ __launch_bounds__(256) void k_var_write(const DevNode *nodes, uint32_t folded, uint64_t n,
                                                   const uint16_t *__restrict__ unit_of, uint32_t W,
                                                   const uint64_t *__restrict__ off, uint8_t *chunk) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gs) {
        const uint64_t o = gld(off + r);
        if (gld(off + r + 1) == o) continue;  // no labels, no record
        uint32_t *rec = reinterpret_cast<uint32_t *>(chunk + 4 * o);
        uint32_t cw = 0, cv = 0;  // the bitmap word being filled
        uint32_t mi = 0, mv = 0;  // mask bytes so far, the word being filled
        (void)emit_row_masks(nodes, folded != 0, (uint32_t)r, [&](uint32_t m, uint32_t, uint32_t d) {
            const uint32_t u = gld(unit_of + d);
            if (u == 0xFFFFu) return;
            if ((u >> 5) != cw) {
                if (cv) gst(rec + cw, cv);
                cw = u >> 5;
                cv = 0;
            }
            cv |= 1u << (u & 31);
            mv |= (m & 0xFFu) << (8 * (mi & 3));
            if ((++mi & 3) == 0) {
                gst(rec + W + mi / 4 - 1, mv);
                mv = 0;
            }
        });
        if (cv) gst(rec + cw, cv);
        if (mi & 3) gst(rec + W + mi / 4, mv);
    }
}

// one thread per directory line of the range
__global__ __launch_bounds__(256) void k_var_lines(const uint64_t *__restrict__ off, const uint16_t *__restrict__ cnt,
                                                   uint64_t n, uint64_t chunk, uint8_t *lines,
                                                   unsigned long long *acc) {
    const uint64_t nl = (n + kLineRows - 1) / kLineRows;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < nl; g += gs) {
        const uint64_t r = g * kLineRows;
        const uint64_t o0 = gld(off + r);
        const uint64_t re = r + kLineRows < n ? r + kLineRows : n;
        const uint64_t span = gld(off + re) - o0;
        if (span >= (1ull << kOffBits)) atomicAdd(acc + 2, 1ull);
        uint32_t e[kLineRows + 1];
        for (uint32_t t = 0; t < kLineRows; ++t)
            e[t] = r + t < n ? (uint32_t)(gld(off + r + t) - o0) | ((uint32_t)gld(cnt + r + t) << kOffBits)
                             : (uint32_t)span;
        e[kLineRows] = (uint32_t)span;
        uint32_t *L = reinterpret_cast<uint32_t *>(lines + g * 64);
        const uint64_t base = chunk + 4 * o0;
        gst(reinterpret_cast<uint64_t *>(L), base);
        for (uint32_t t = 0; t <= kLineRows; ++t) gst(L + 2 + t, e[t]);
    }
}

int build_grid(uint64_t items) { return (int)std::max<uint64_t>(1, std::min<uint64_t>((items + 255) / 256, 65536)); }

struct U16ToU64 {
    __host__ __device__ __forceinline__ uint64_t operator()(const uint16_t &x) const { return x; }
};

}  // namespace

int var_build_range(RowsImage &im, const Ctx &range, uint64_t row0, VarScratch &ws, hipStream_t s) {
    const uint64_t nr = range.tree.num_rows;
    if (row0 % kLineRows) {
        set_error("variable-length records: range not aligned to a directory line");
        return MBRWT_ERR_INVALID;
    }
    int rc;
    if ((rc = ensure(ws.units, (nr + 1) * 2)) || (rc = ensure(ws.cnt, (nr + 1) * 2)) ||
        (rc = ensure(ws.off, (nr + 1) * 8)) || (rc = ensure(ws.acc, 64)))
        return rc;
    uint16_t *d_units = reinterpret_cast<uint16_t *>(ws.units.buf);
    uint16_t *d_cnt = reinterpret_cast<uint16_t *>(ws.cnt.buf);
    uint64_t *d_off = reinterpret_cast<uint64_t *>(ws.off.buf);
    unsigned long long *d_acc = reinterpret_cast<unsigned long long *>(ws.acc.buf);
    if (!im.d_unit_of) {
        MBRWT_HIP(hipMalloc(&im.d_unit_of, im.var_unit_of.size() * 2));
        MBRWT_HIP(hipMemcpy(im.d_unit_of, im.var_unit_of.data(), im.var_unit_of.size() * 2, hipMemcpyHostToDevice));
    }
    MBRWT_HIP(hipMemsetAsync(d_acc, 0, 64, s));
    MBRWT_HIP(hipMemsetAsync(d_units + nr, 0, 2, s));
    hipLaunchKernelGGL(k_var_measure, dim3(build_grid(nr)), dim3(256), 0, s, range.d_nodes, range.tree.folded ? 1u : 0u,
                       nr, im.d_unit_of, im.var_W, d_units, d_cnt, d_acc);
    MBRWT_HIP(hipGetLastError());
    hipcub::TransformInputIterator<uint64_t, U16ToU64, const uint16_t *> it(d_units, U16ToU64());
    size_t sb = 0;
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, sb, it, d_off, nr + 1, s));
    if ((rc = ensure(ws.scan, sb))) return rc;
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(ws.scan.buf, sb, it, d_off, nr + 1, s));
    unsigned long long h[3];
    uint64_t units = 0;
    MBRWT_HIP(hipMemcpyAsync(h, d_acc, sizeof(h), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipMemcpyAsync(&units, d_off + nr, 8, hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (h[2]) {
        set_error("variable-length records: a row outside the unit layout");
        return MBRWT_ERR_UNSUPPORTED;
    }
    if (h[0] != range.tree.num_relations) {
        set_error("variable-length records: label count differs from the node image");
        return MBRWT_ERR_DEVICE;
    }
    // this range's records: their own allocation (+ a line of padding for
    // the decoder's whole 16-byte chunks)
    void *chunk = nullptr;
    const uint64_t bytes = 4 * units + 64;
    MBRWT_HIP(hipMalloc(&chunk, bytes));
    im.var_chunks.push_back(chunk);
    im.var_rec_bytes += 4 * units;
    im.record_bytes += 4 * units;
    MBRWT_HIP(hipMemsetAsync(chunk, 0, bytes, s));
    hipLaunchKernelGGL(k_var_write, dim3(build_grid(nr)), dim3(256), 0, s, range.d_nodes, range.tree.folded ? 1u : 0u,
                       nr, im.d_unit_of, im.var_W, d_off, reinterpret_cast<uint8_t *>(chunk));
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipMemsetAsync(d_acc, 0, 64, s));
    hipLaunchKernelGGL(k_var_lines, dim3(build_grid((nr + kLineRows - 1) / kLineRows)), dim3(256), 0, s, d_off, d_cnt,
                       nr, (uint64_t)(uintptr_t)chunk, im.var_lines + (row0 / kLineRows) * 64, d_acc);
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipMemcpyAsync(h, d_acc, sizeof(h), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (h[2]) {
        set_error("variable-length records: 13 records longer than 512 KiB");
        return MBRWT_ERR_UNSUPPORTED;
    }
    return MBRWT_OK;
}

// measure only (the first range's layout decision): record bytes and labels
int var_measure_range(RowsImage &im, const Ctx &range, VarScratch &ws, uint64_t *rec_bytes, hipStream_t s) {
    const uint64_t nr = range.tree.num_rows;
    int rc;
    if ((rc = ensure(ws.units, (nr + 1) * 2)) || (rc = ensure(ws.cnt, (nr + 1) * 2)) || (rc = ensure(ws.acc, 64)))
        return rc;
    if (!im.d_unit_of) {
        MBRWT_HIP(hipMalloc(&im.d_unit_of, im.var_unit_of.size() * 2));
        MBRWT_HIP(hipMemcpy(im.d_unit_of, im.var_unit_of.data(), im.var_unit_of.size() * 2, hipMemcpyHostToDevice));
    }
    unsigned long long *d_acc = reinterpret_cast<unsigned long long *>(ws.acc.buf);
    MBRWT_HIP(hipMemsetAsync(d_acc, 0, 64, s));
    hipLaunchKernelGGL(k_var_measure, dim3(build_grid(nr)), dim3(256), 0, s, range.d_nodes, range.tree.folded ? 1u : 0u,
                       nr, im.d_unit_of, im.var_W, reinterpret_cast<uint16_t *>(ws.units.buf),
                       reinterpret_cast<uint16_t *>(ws.cnt.buf), d_acc);
    MBRWT_HIP(hipGetLastError());
    unsigned long long h[3];
    MBRWT_HIP(hipMemcpyAsync(h, d_acc, sizeof(h), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (h[2]) {
        set_error("variable-length records: a row outside the unit layout");
        return MBRWT_ERR_UNSUPPORTED;
    }
    *rec_bytes = h[1];
    return MBRWT_OK;
}

void var_free_scratch(VarScratch &ws) {
    for (Workspace *w : {&ws.units, &ws.cnt, &ws.off, &ws.acc, &ws.scan})
        if (w->buf) (void)hipFree(w->buf);
    ws = VarScratch();
}

// ------------------------------------------------------------------------
// queries
// ------------------------------------------------------------------------
namespace {

struct VarView {
    uint64_t lines, magic, num_rows;
    uint32_t W;
};
__device__ __forceinline__ uint64_t var_line(uint64_t r, uint64_t magic) { return __umul64hi(r, magic); }
// row r's record: address, length in 4-byte units, label count
__device__ __forceinline__ void var_locate(const VarView &v, uint64_t r, uint64_t &addr, uint32_t &len,
                                           uint32_t &count) {
    const uint64_t g = var_line(r, v.magic);
    const uint32_t t = (uint32_t)(r - g * kLineRows);
    const uint64_t L = v.lines + g * 64;
    const uint64_t base = gld_at<uint64_t>(L);
    const uint32_t e0 = gld_at<uint32_t>(L + 8 + 4 * t), e1 = gld_at<uint32_t>(L + 12 + 4 * t);
    const uint32_t o0 = e0 & ((1u << kOffBits) - 1), o1 = e1 & ((1u << kOffBits) - 1);
    count = e0 >> kOffBits;
    len = o1 - o0;
    addr = base + 4ull * o0;
}

// one lane's labels of a record: from bitmap word wi (its bits below the
// lane's first unit already cleared: w) and mask byte `cur` on, nlab labels;
// emit(k, label) for its k-th label.  Word(i) / Byte(i) read the record.
// (The refill of an exhausted mask runs in ~88 % of the iterations at the
// RefSeq shape -- 1.13 labels per reached unit -- so it is computed
// unconditionally and selected, rather than branched over; only the step
// to the next bitmap word, rare, is a branch.)
template <class Word, class Byte, class Base, class Emit>
__device__ __forceinline__ void var_lane_labels(Word word, Byte byte, uint32_t wi, uint32_t w, uint32_t cur,
                                                uint32_t nlab, Base ubase, Emit emit) {
    uint32_t m = 0, base = 0;
    for (uint32_t k = 0; k < nlab; ++k) {
        const bool rf = m == 0;
        if (rf && w == 0) {
            do {
                w = word(++wi);
            } while (w == 0);
        }
        const uint32_t u = wi * 32 + (uint32_t)__builtin_ctz(w | (rf ? 0u : 0x80000000u));
        const uint32_t nb = ubase(u), nm = byte(cur);
        base = rf ? nb : base;
        m = rf ? nm : m;
        w = rf ? (w & (w - 1)) : w;
        cur += rf ? 1u : 0u;
        emit(k, base + (uint32_t)__builtin_ctz(m));
        m &= m - 1;
    }
}

// the labels of `items` consecutive unit masks starting at mask byte `b0`
// (aligned 32-bit reads, the partial words masked)
template <class Word>
__device__ __forceinline__ uint32_t var_mask_labels(Word word, uint32_t byte0, uint32_t items) {
    if (!items) return 0;
    const uint32_t b1 = byte0 + items;
    uint32_t labs = 0;
    for (uint32_t wb = byte0 & ~3u; wb < b1; wb += 4) {
        uint32_t v = word(wb >> 2);
        if (wb < byte0) v &= ~0u << (8 * (byte0 - wb));
        if (wb + 4 > b1) v &= ~0u >> (8 * (wb + 4 - b1));
        labs += (uint32_t)__builtin_popcount(v);
    }
    return labs;
}

struct VarParams {
    const uint64_t *rows;
    uint64_t n;
    VarView v;
    uint64_t *loc;                // per batch row: record address | length in 4-byte units << 48
    uint32_t *cnt;                // per batch row: label count (n + 1 entries; cnt[n] = 0)
    const uint64_t *offsets;      // the CSR offsets (the scan of cnt)
    uint32_t *cols;
    uint64_t cap;
    const uint32_t *units;        // per unit: first column | arity << 16
    uint32_t U;
    uint32_t CR, CS;              // per wave: record bytes, stage labels (LDS)
    uint32_t ustride;             // unit u's first column = u * ustride (0: the unit table)
    unsigned long long *scalars;  // [2] error flags (bit 0: row out of range)
    unsigned long long *status;   // the call's {needed, status, sticky}
};

__global__ __launch_bounds__(256) void k_var_locate(VarParams p) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i0 == 0) p.status[1] = MBRWT_OK;  // k_var_decode raises it
    for (uint64_t i = i0; i <= p.n; i += gs) {
        if (i == p.n) {
            gst(p.cnt + i, 0u);
            continue;
        }
        const uint64_t row = gld(p.rows + i);
        uint64_t addr = 0;
        uint32_t len = 0, count = 0;
        if (row < p.v.num_rows) {
            var_locate(p.v, row, addr, len, count);
        } else {
            atomicOr(&p.scalars[2], 1ull);
        }
        gst(p.loc + i, addr | (uint64_t)len << 48);
        gst(p.cnt + i, count);
    }
}

__device__ __forceinline__ void var_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void var_publish(unsigned long long *status, uint64_t st) {
    atomicMax(&status[1], (unsigned long long)st);
    atomicOr(&status[2], 1ull << st);
}

// k_var_decode: R = 64 / G rows per tile (one wave), G lanes per row; the
// grid is persistent, WPB waves per workgroup share the unit table in LDS.
// (G >= 8: tiles of <= 8 rows need < 6 KB of LDS per wave, so 24 waves per
// CU fit when the registers do: 6 waves per SIMD requested, 79 VGPRs, no
// scratch; G <= 4 is bound by LDS at 16 waves per CU anyway.)
template <int G, int WPB>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(G >= 8 ? 6 : 1))) void k_var_decode(VarParams p) {
    constexpr uint32_t R = 64 / G;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_var[];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t n = p.n;
    const uint64_t total_all = gld(p.offsets + n);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const uint64_t err = p.scalars[2];
        p.scalars[2] = 0;
        p.status[0] = total_all;
        var_publish(p.status, (err & 1) ? MBRWT_ERR_RANGE : total_all > p.cap ? MBRWT_ERR_CAPACITY : MBRWT_OK);
    }
    if (total_all > p.cap) return;
    AS_LDS uint16_t *ubase = (AS_LDS uint16_t *)lds_var;
    for (uint32_t i = threadIdx.x; i < p.U; i += blockDim.x) ubase[i] = (uint16_t)(gld(p.units + i) & 0xFFFFu);
    // (speculative reads may index up to 31 entries past the last unit)
    __syncthreads();
    const uint32_t ub_words = ((p.U + 32) * 2 + 15) / 16 * 4;  // (16-byte aligned; 32 entries of slack)
    const uint32_t per_wave = p.CR + p.CR / 16 + 2 * p.CS;
    AS_LDS uint8_t *wb = (AS_LDS uint8_t *)(lds_var + ub_words) + wv * per_wave;
    AS_LDS uint8_t *rec = wb;                                   // CR bytes of 16-byte chunks
    AS_LDS uint8_t *owner = wb + p.CR;                          // CR / 16 chunk owners (row in the tile)
    AS_LDS uint16_t *stage = (AS_LDS uint16_t *)(owner + p.CR / 16);  // CS labels
    const uint32_t rr = lane / G, q = lane % G;
    const uint32_t W = p.v.W;
    const uint32_t Wq = (W + G - 1) / G, w0 = q * Wq, w1 = w0 + Wq < W ? w0 + Wq : W;
    const uint64_t ntiles = (n + R - 1) / R;
    const uint64_t tstride = (uint64_t)gridDim.x * WPB;
    for (uint64_t t = (uint64_t)blockIdx.x * WPB + wv; t < ntiles; t += tstride) {
        const uint64_t r0 = t * R;
        const uint32_t nr = (uint32_t)(n - r0 < R ? n - r0 : R);
        const bool in = rr < nr;
        const uint64_t lc = in ? gld(p.loc + r0 + rr) : 0;
        const uint32_t count = in ? gld(p.cnt + r0 + rr) : 0u;
        const uint64_t roff = gld(p.offsets + r0 + (in ? rr : nr));
        const uint64_t tbase = (uint64_t)__shfl((unsigned long long)roff, 0, 64);
        const uint64_t tend = gld(p.offsets + r0 + nr);
        const uint32_t ttot = (uint32_t)(tend - tbase);
        const uint64_t addr = lc & ((1ull << 48) - 1);
        const uint32_t len = (uint32_t)(lc >> 48);
        // the tile's records as 16-byte chunks: lane q == 0 of each row
        // counts its row's chunks, a wave scan numbers them
        const uint64_t first = addr >> 4;
        uint32_t nch = (q == 0 && in && count) ? (uint32_t)(((addr + 4ull * len - 1) >> 4) - first + 1) : 0u;
        uint32_t x = nch;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
            if (lane >= d) x += y;
        }
        const uint32_t TC = __builtin_amdgcn_readlane(x, 63);
        const uint32_t cs = x - nch;  // this row's first chunk (valid on lane q == 0)
        const uint32_t cs_row = (uint32_t)__shfl((int)cs, (int)(rr * G), 64);
        const bool fits = TC * 16 <= p.CR && ttot <= p.CS;
        if (fits) {
            for (uint32_t k = 0; k < nch; ++k) owner[cs + k] = (uint8_t)rr;
            var_wave_sync();
            // coalesced gather: lane g of round k loads chunk 64 k + g
            for (uint32_t g0 = 0; g0 < TC; g0 += 256) {
                u32x4_t v[4];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint32_t g = g0 + 64 * j + lane;
                    const uint32_t o = g < TC ? owner[g] : 0u;
                    const uint32_t fl = (uint32_t)__shfl((int)(uint32_t)first, (int)(o * G), 64);
                    const uint32_t fh = (uint32_t)__shfl((int)(uint32_t)(first >> 32), (int)(o * G), 64);
                    const uint32_t co = (uint32_t)__shfl((int)cs, (int)(o * G), 64);
                    if (g < TC) v[j] = gld_at<u32x4_t>(((((uint64_t)fh << 32) | fl) + (g - co)) << 4);
                }
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint32_t g = g0 + 64 * j + lane;
                    if (g < TC) ((AS_LDS u32x4_t *)rec)[g] = v[j];
                }
            }
            var_wave_sync();
        }
        // this lane's share of the row: an equal share of its units (mask
        // bytes), found from the units in words [w0, w1) of every lane
        const AS_LDS uint8_t *rl = rec + 16 * cs_row + (uint32_t)(addr & 15);
        auto word_l = [&](uint32_t i) -> uint32_t { return *(const AS_LDS uint32_t *)(rl + 4 * i); };
        auto byte_l = [&](uint32_t i) -> uint32_t { return rl[i]; };
        auto word_g = [&](uint32_t i) -> uint32_t { return gld_at<uint32_t>(addr + 4ull * i); };
        auto byte_g = [&](uint32_t i) -> uint32_t { return gld_at<uint8_t>(addr + i); };
        auto word_a = [&](uint32_t i) -> uint32_t { return fits ? word_l(i) : word_g(i); };
        uint32_t items = 0;
        if (count)
            for (uint32_t i = w0; i < w1; ++i) items += (uint32_t)__builtin_popcount(word_a(i));
        uint32_t wi = 0, wv0 = 0, j0 = 0, nunits = 0;
        if constexpr (G == 1) {
            wi = 0;
            wv0 = count ? word_a(0) : 0u;
            nunits = items;
        } else {
            // units of the word ranges before this lane's (inclusive scan - own)
            uint32_t ie = items;
#pragma unroll
            for (uint32_t d = 1; d < (uint32_t)G; d <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)ie, d, 64);
                if (q >= d) ie += y;
            }
            const uint32_t NB = (uint32_t)__shfl((int)ie, (int)(rr * G + G - 1), 64);  // the row's units
            j0 = q * NB / G;
            nunits = (q + 1) * NB / G - j0;
            // the word range holding unit j0: after every range ending at or before it
            uint32_t qs = 0, before = 0;
#pragma unroll
            for (uint32_t g = 0; g < (uint32_t)G; ++g) {
                const uint32_t e = (uint32_t)__shfl((int)ie, (int)(rr * G + g), 64);
                if (e <= j0) {
                    qs = g + 1;
                    before = e;
                }
            }
            // unit j0 is unit k of that range: scan its words, then select
            uint32_t k = j0 - before;
            wi = qs * Wq;
            if (nunits) {
                uint32_t w = word_a(wi);
                for (uint32_t c = (uint32_t)__builtin_popcount(w); k >= c; c = (uint32_t)__builtin_popcount(w)) {
                    k -= c;
                    w = word_a(++wi);
                }
                // clear the k lowest set bits
                for (; k; --k) w &= w - 1u;
                wv0 = w;
            }
        }
        const uint32_t labs = fits ? var_mask_labels(word_l, 4 * W + j0, nunits) : var_mask_labels(word_g, 4 * W + j0, nunits);
        uint32_t lb = labs;
#pragma unroll
        for (uint32_t d = 1; d < (uint32_t)G; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)lb, d, 64);
            if (q >= d) lb += y;
        }
        lb -= labs;
        const uint32_t pos = (uint32_t)(roff - tbase) + lb;  // the lane's first label in the tile
        if (fits) {
            const uint32_t us = p.ustride;
            // (r05: mask bytes read as words and labels stored in pairs halved
            // the LDS bank-conflict cycles, 218 M -> 108 M per 10 M rows, but
            // added 17 % VALU: 2.46 against 2.22 ms; profiles/r05/v06_*)
            if (us && !(us & (us - 1))) {  // (a shift: v_mul_lo_u32 issues at a quarter rate)
                const uint32_t sh = (uint32_t)__builtin_ctz(us);
                var_lane_labels(word_l, byte_l, wi, wv0, 4 * W + j0, labs, [&](uint32_t u) -> uint32_t { return u << sh; },
                                [&](uint32_t k, uint32_t lab) { stage[pos + k] = (uint16_t)lab; });
            } else if (us)
                var_lane_labels(word_l, byte_l, wi, wv0, 4 * W + j0, labs, [&](uint32_t u) -> uint32_t { return u * us; },
                                [&](uint32_t k, uint32_t lab) { stage[pos + k] = (uint16_t)lab; });
            else
                var_lane_labels(word_l, byte_l, wi, wv0, 4 * W + j0, labs,
                                [&](uint32_t u) -> uint32_t { return ubase[u]; },
                                [&](uint32_t k, uint32_t lab) { stage[pos + k] = (uint16_t)lab; });
            var_wave_sync();
            // the tile's labels: contiguous in the CSR, 4 per lane and store
            uint32_t *dst = p.cols + tbase;
            for (uint32_t i = 4 * lane; i < ttot; i += 256) {
                if (i + 4 <= ttot) {
                    // one 8-byte LDS read per 4 labels (r05: the same LDS instruction
                    // count and conflicts as four u16 reads -- the compiler merged
                    // those already -- 2.150 vs 2.155 ms, profiles/r05/v11_*)
                    const uint64_t w4 = *(const AS_LDS uint64_t *)(stage + i);
                    const uint32_t lo = (uint32_t)w4, hi = (uint32_t)(w4 >> 32);
                    *(AS_GLOBAL u32x4_t *)(uintptr_t)(dst + i) = u32x4_t{lo & 0xFFFFu, lo >> 16, hi & 0xFFFFu, hi >> 16};
                } else {
                    for (uint32_t j = i; j < ttot; ++j) gst(dst + j, (uint32_t)stage[j]);
                }
            }
            var_wave_sync();  // the stage, the chunks and the owners are reused
        } else {
            // a tile beyond the LDS budget: records read and labels stored
            // straight from / to global memory
            uint32_t *dst = p.cols + tbase + pos;
            var_lane_labels(word_g, byte_g, wi, wv0, 4 * W + j0, labs, [&](uint32_t u) -> uint32_t { return ubase[u]; },
                            [&](uint32_t k, uint32_t lab) { gst(dst + k, lab); });
        }
    }
}

// one row's labels from the records in global memory (point / count /
// column queries)
template <class Leaf>
__device__ __forceinline__ void var_row(const VarView &v, const uint32_t *units, uint64_t row, Leaf leaf) {
    uint64_t addr;
    uint32_t len, count;
    var_locate(v, row, addr, len, count);
    if (!count) return;
    var_lane_labels([&](uint32_t i) -> uint32_t { return gld_at<uint32_t>(addr + 4ull * i); },
                    [&](uint32_t i) -> uint32_t { return gld_at<uint8_t>(addr + i); }, 0u,
                    gld_at<uint32_t>(addr), 4 * v.W, count,
                    [&](uint32_t u) -> uint32_t { return gld(units + u) & 0xFFFFu; },
                    [&](uint32_t, uint32_t lab) { leaf(lab); });
}

__global__ __launch_bounds__(256) void k_var_get(VarView v, const uint32_t *units, const uint64_t *rows,
                                                 const uint64_t *qcols, uint64_t n, uint64_t num_cols, uint8_t *out,
                                                 unsigned long long *scalars) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const uint64_t row = gld(rows + i), col = gld(qcols + i);
        if (row >= v.num_rows || col >= num_cols) {
            atomicOr(&scalars[2], 1ull);
            gst(out + i, (uint8_t)0);
            continue;
        }
        uint32_t hit = 0;
        var_row(v, units, row, [&](uint32_t c) { hit |= c == col; });
        gst(out + i, (uint8_t)hit);
    }
}

// count_labels (annotate_static.cpp:149-162) and the V / L accounting
// (V = 1 + the arities of the internal nodes the descent
// reaches).  A unit's ancestors at levels 0..K-1 come from `anc`; an
// ancestor is newly reached where it differs from the previous unit's.
template <bool WORK>
__global__ __launch_bounds__(256) void k_var_count(VarView v, const uint32_t *units, const uint32_t *anc, uint32_t K,
                                                   const DevNode *nodes, const uint64_t *rows, uint64_t n,
                                                   unsigned long long *counts, unsigned long long *scalars) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long vis = 0, lab = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const uint64_t row = gld(rows + i);
        if (row >= v.num_rows) {
            atomicOr(&scalars[2], 1ull);
            continue;
        }
        vis += 1;
        if constexpr (WORK) {
            uint64_t addr;
            uint32_t len, count;
            var_locate(v, row, addr, len, count);
            if (!count) continue;
            lab += count;
            uint32_t prev = 0xFFFFFFFFu;
            for (uint32_t wi = 0; wi < v.W; ++wi)
                for (uint32_t w = gld_at<uint32_t>(addr + 4ull * wi); w; w &= w - 1) {
                    const uint32_t u = wi * 32 + (uint32_t)__builtin_ctz(w);
                    vis += (gld(units + u) >> 16) & 0xFFu;  // the leaf parent's mask
                    for (uint32_t k = 0; k < K; ++k) {      // its ancestors new to this row
                        const uint32_t a = gld(anc + (uint64_t)u * K + k);
                        if (prev == 0xFFFFFFFFu || gld(anc + (uint64_t)prev * K + k) != a) vis += gld(nodes + a).arity;
                    }
                    prev = u;
                }
        } else {
            var_row(v, units, row, [&](uint32_t c) { atomicAdd(counts + c, 1ull); });
        }
    }
    if constexpr (WORK) {
        for (int off = 32; off > 0; off >>= 1) {
            vis += __shfl_down(vis, off);
            lab += __shfl_down(lab, off);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&scalars[3], vis);
            atomicAdd(&scalars[4], lab);
        }
    }
}

struct VarHasColumn {
    VarView v;
    const uint32_t *units;
    uint32_t col;
    __device__ bool operator()(const uint64_t &row) const {
        bool hit = false;
        var_row(v, units, row, [&](uint32_t c) { hit |= c == col; });
        return hit;
    }
};
struct VarHasColumnCount {
    VarHasColumn f;
    __device__ uint64_t operator()(const uint64_t &row) const { return f(row) ? 1u : 0u; }
};

VarView var_view(const Ctx &c) {
    VarView v;
    v.lines = (uint64_t)(uintptr_t)c.rows.var_lines;
    v.magic = (uint64_t)((((unsigned __int128)1) << 64) / kLineRows) + 1;
    v.num_rows = c.tree.num_rows;
    v.W = c.rows.var_W;
    return v;
}

struct U32ToU64v {
    __host__ __device__ __forceinline__ uint64_t operator()(const uint32_t &x) const { return x; }
};

using VarFn = void (*)(VarParams);
constexpr uint32_t kVarWpb = 4;
VarFn var_fn(uint32_t G) {
    return G == 1    ? k_var_decode<1, kVarWpb>
           : G == 2  ? k_var_decode<2, kVarWpb>
           : G == 4  ? k_var_decode<4, kVarWpb>
           : G == 8  ? k_var_decode<8, kVarWpb>
                     : k_var_decode<16, kVarWpb>;
}

uint64_t simple_grid(uint64_t n) { return std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 65536)); }

}  // namespace

// lanes per row and the per-wave LDS budget from the image's statistics
// (labels and record bytes per row), within the workgroup's LDS: the unit
// table (u16 per unit) is staged once per workgroup, so a tree with many
// units leaves less for the kWpb waves' record / owner / stage areas, which
// are then scaled down (tiles beyond them take the global path; at worst
// CR = CS = 0 and every non-empty tile does).  lds_ok: a mean tile still fits
// (the build declines the variable-length records otherwise).
constexpr size_t kVarLdsMax = 160u << 10;  // gfx950: LDS per CU, all of it one workgroup's at most
struct VarGeom {
    uint32_t G, CR, CS;
    bool lds_ok;
};
static VarGeom var_geometry_of(uint32_t var_G, uint32_t U, double lab, double rec) {
    VarGeom g{};
    g.G = var_G ? var_G : lab >= 48.0 ? 4u : lab >= 12.0 ? 2u : 1u;
    const double R = 64.0 / g.G;
    // a tile's records (whole 16-byte chunks: + 16 per row) and labels with
    // ~6 standard deviations of room; larger tiles take the global path
    const double cr = R * (rec + 16.0) + 6.0 * std::sqrt(R) * (rec * 0.25 + 16.0) + 256.0;
    const double cs = R * lab + 6.0 * std::sqrt(R * lab + 1.0) * 2.0 + 64.0;
    g.CR = (uint32_t)std::min(32768.0, std::ceil(cr / 256.0) * 256.0);
    g.CS = (uint32_t)std::min(16384.0, std::ceil(cs / 64.0) * 64.0);
    const size_t ub = ((size_t)(U + 32) * 2 + 15) / 16 * 16;
    const size_t avail = ub < kVarLdsMax ? (kVarLdsMax - ub) / kVarWpb : 0;
    auto need = [&]() { return (size_t)g.CR + g.CR / 16 + 2ull * g.CS; };
    if (need() > avail) {
        const double f = (double)avail / (double)need();
        g.CR = (uint32_t)(std::floor(g.CR * f / 256.0) * 256.0);
        g.CS = (uint32_t)(std::floor(g.CS * f / 64.0) * 64.0);
        while (need() > avail && (g.CR || g.CS)) {
            if (g.CR) g.CR -= 256;
            if (need() > avail && g.CS) g.CS -= 64;
        }
    }
    g.lds_ok = g.CR >= R * (rec + 16.0) && g.CS >= R * lab;
    return g;
}
static void var_geometry(const Ctx &c, uint32_t &G, uint32_t &CR, uint32_t &CS) {
    const RowsImage &im = c.rows;
    const double rows = std::max<double>(1.0, (double)c.tree.num_rows);
    const VarGeom g = var_geometry_of(im.var_G, (uint32_t)im.var_units.size(), (double)c.tree.num_relations / rows,
                                      (double)im.var_rec_bytes / rows);
    G = g.G;
    CR = g.CR;
    CS = g.CS;
}
bool var_lds_fits(const RowsImage &im, double labels_per_row, double record_bytes_per_row) {
    return var_geometry_of(im.var_G, (uint32_t)im.var_units.size(), labels_per_row, record_bytes_per_row).lds_ok;
}

int var_get_rows(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets, uint32_t *d_cols, uint64_t cap,
                 uint64_t *needed, hipStream_t s, uint64_t *d_status) {
    const RowsImage &im = c.rows;
    if (n > 0x7FFFFFF0ull) {
        set_error("batch larger than 2^31 rows");
        return MBRWT_ERR_UNSUPPORTED;
    }
    int rc;
    // ws_temp: loc (n x u64) | cnt ((n + 1) x u32); ws_counts: the kernel's counters
    const uint64_t cnt_at = n * 8;
    if ((rc = ensure(c.ws_temp, cnt_at + (n + 1) * 4 + 16))) return rc;
    const bool fresh = c.ws_counts.bytes < 64;
    if ((rc = ensure(c.ws_counts, 64))) return rc;
    unsigned long long *d_sc = reinterpret_cast<unsigned long long *>(c.ws_counts.buf);
    if (fresh || c.rows_sc_dirty || c.rows_sc_at != 0) {
        MBRWT_HIP(hipMemsetAsync(d_sc, 0, 32, s));
        c.rows_sc_dirty = false;
        c.rows_sc_at = 0;
    }
    uint64_t *d_loc = reinterpret_cast<uint64_t *>(c.ws_temp.buf);
    uint32_t *d_cnt = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(c.ws_temp.buf) + cnt_at);
    hipcub::TransformInputIterator<uint64_t, U32ToU64v, const uint32_t *> it(d_cnt, U32ToU64v());
    size_t sb = 0;
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, sb, it, d_offsets, n + 1, s));
    if ((rc = ensure(c.ws_scan, sb))) return rc;
    unsigned long long *st_blk = reinterpret_cast<unsigned long long *>(d_status ? d_status : c.d_scalars);

    uint32_t G, CR, CS;
    var_geometry(c, G, CR, CS);
    VarParams p{};
    p.rows = d_rows;
    p.n = n;
    p.v = var_view(c);
    p.loc = d_loc;
    p.cnt = d_cnt;
    p.offsets = d_offsets;
    p.cols = d_cols;
    p.cap = cap;
    p.units = im.d_var_units;
    p.U = (uint32_t)im.var_units.size();
    p.CR = CR;
    p.CS = CS;
    p.ustride = im.var_ustride;
    p.scalars = d_sc;
    p.status = st_blk;
    const VarFn kfn = var_fn(G);
    const size_t lds = ((p.U + 32) * 2 + 15) / 16 * 16 + kVarWpb * (size_t)(CR + CR / 16 + 2 * CS);
    const uint32_t threads = 64 * kVarWpb;
    if (c.rb_fn != reinterpret_cast<const void *>(kfn) || c.rb_lds != lds || c.rb_threads != threads) {
        if (lds > 65536)
            MBRWT_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kfn),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        int dev_cus = 0, per_cu = 0;
        (void)hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, c.device);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(kfn), threads, lds) !=
                hipSuccess ||
            per_cu <= 0)
            per_cu = 1;
        if (im.occ_cap) per_cu = std::min<int>(per_cu, (int)im.occ_cap);
        c.rb_fn = reinterpret_cast<const void *>(kfn);
        c.rb_lds = lds;
        c.rb_threads = threads;
        c.rb_cap = 0;
        c.rb_blocks = std::max(1, dev_cus) * per_cu;
    }
    c.rows_sc_dirty = true;  // until k_var_decode has run
    hipEvent_t e0 = c.ev0, e1 = c.ev1;
    if (c.timing && d_status) {
        if (c.async_ev.size() <= c.async_used) {
            hipEvent_t ea = nullptr, eb = nullptr;
            MBRWT_HIP(hipEventCreate(&ea));
            MBRWT_HIP(hipEventCreate(&eb));
            c.async_ev.push_back({ea, eb});
        }
        e0 = c.async_ev[c.async_used].first;
        e1 = c.async_ev[c.async_used].second;
        ++c.async_used;
    }
    hipLaunchKernelGGL(k_var_locate, dim3((unsigned)simple_grid(n + 1)), dim3(256), 0, s, p);
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(c.ws_scan.buf, sb, it, d_offsets, n + 1, s));
    if (c.timing) MBRWT_HIP(hipEventRecord(e0, s));
    {
        const uint64_t R = 64 / G, nt = (n + R - 1) / R;
        // (persistent: one tile per wave, as k_traverse_rows, measured 1.4 %
        // slower here -- 2.215 vs 2.185 ms per 10 M rows at C3, profiles/r05)
        const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>((nt + kVarWpb - 1) / kVarWpb, (uint64_t)c.rb_blocks));
        hipLaunchKernelGGL(kfn, dim3((unsigned)g), dim3(threads), lds, s, p);
        MBRWT_HIP(hipGetLastError());
    }
    if (c.timing) MBRWT_HIP(hipEventRecord(e1, s));
    c.rows_sc_dirty = false;
    if (d_status) return MBRWT_OK;
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (c.timing) {
        float ms = 0;
        MBRWT_HIP(hipEventElapsedTime(&ms, c.ev0, c.ev1));
        c.timing_ms += ms;
        c.timing_launches += 1;
    }
    const uint64_t total = c.h_scalars[0], st = c.h_scalars[1];
    if (needed) *needed = total;
    switch (st) {
        case MBRWT_OK: return MBRWT_OK;
        case MBRWT_ERR_RANGE: set_error("row out of range"); return MBRWT_ERR_RANGE;
        case MBRWT_ERR_CAPACITY: set_error("cols_cap too small"); return MBRWT_ERR_CAPACITY;
        default: set_error("variable-length record decode failed"); return MBRWT_ERR_DEVICE;
    }
}

int var_get_batch(Ctx &c, const uint64_t *d_rows, const uint64_t *d_cols, uint64_t n, uint8_t *d_out, hipStream_t s) {
    if (n == 0) return MBRWT_OK;
    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 8 * sizeof(uint64_t), s));
    hipLaunchKernelGGL(k_var_get, dim3((unsigned)simple_grid(n)), dim3(256), 0, s, var_view(c),
                       (const uint32_t *)c.rows.d_var_units, d_rows, d_cols, n, c.tree.num_columns, d_out,
                       reinterpret_cast<unsigned long long *>(c.d_scalars));
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    return (c.h_scalars[2] & 1) ? MBRWT_ERR_RANGE : MBRWT_OK;
}

int var_count(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_counts, uint64_t *visits, uint64_t *labels,
              hipStream_t s) {
    const bool work = d_counts == nullptr;
    if (!work && c.tree.num_columns)
        MBRWT_HIP(hipMemsetAsync(d_counts, 0, c.tree.num_columns * sizeof(uint64_t), s));
    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 8 * sizeof(uint64_t), s));
    if (n) {
        auto fn = work ? k_var_count<true> : k_var_count<false>;
        hipLaunchKernelGGL(fn, dim3((unsigned)simple_grid(n)), dim3(256), 0, s, var_view(c),
                           (const uint32_t *)c.rows.d_var_units, (const uint32_t *)c.rows.d_var_anc, c.rows.uni,
                           (const DevNode *)c.d_nodes, d_rows, n, reinterpret_cast<unsigned long long *>(d_counts),
                           reinterpret_cast<unsigned long long *>(c.d_scalars));
    }
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (c.h_scalars[2] & 1) return MBRWT_ERR_RANGE;
    if (visits) *visits = c.h_scalars[3];
    if (labels) *labels = c.h_scalars[4];
    return MBRWT_OK;
}

int var_get_column(Ctx &c, uint64_t column, uint64_t *d_rows, uint64_t rows_cap, uint64_t *rows_needed,
                   hipStream_t s) {
    if (column >= c.tree.num_columns) {
        set_error("column out of range");
        return MBRWT_ERR_RANGE;
    }
    const uint64_t n = c.tree.num_rows;
    const VarHasColumn f{var_view(c), c.rows.d_var_units, (uint32_t)column};
    hipcub::CountingInputIterator<uint64_t> rows_it(0);
    hipcub::TransformInputIterator<uint64_t, VarHasColumnCount, hipcub::CountingInputIterator<uint64_t>> cnt_it(
        rows_it, VarHasColumnCount{f});
    int rc;
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

// shards.hip -- rows >= 2^32 (the reference's Row is uint64_t,
// binary_matrix.hpp:11).
//
// Every position inside one device image is u32 (PLANE rank words, PACK2 /
// PACKT block indices).  A BRWT restricted to a row range [a, b) is again a
// BRWT: the root keeps its bits over [a, b), and a child of node u keeps its
// bits over [rank1(u, lo_u), rank1(u, hi_u)) -- the positions of u's set bits
// inside u's range (BRWT.cpp:30,43: a child's row space is its parent's set
// positions).  So a context over more than 2^32 rows holds K sub-contexts of
// shard_rows rows each, built by the ordinary builders, and a query batch is
// routed: the rows are grouped by shard with a stable radix sort of their
// shard ids, each shard answers its group with its own kernels (local rows =
// row - shard start), and the per-shard CSRs are scattered back into the
// batch's order.  Results are the reference's get_row over the whole matrix.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "mbrwt_internal.hpp"

namespace mbrwt {

uint64_t shard_rows_for(uint64_t num_rows) {
    // MBRWT_BUILD_SHARD_ROWS: test hook (small shards exercise the routing on
    // oracle-sized trees); otherwise shards only when one image cannot hold the rows
    if (const uint64_t v = build_tuning().shard_rows; v > 0 && v < num_rows) return std::min<uint64_t>(v, kShardRowsMax);
    return num_rows > kMaxRows ? kShardRowsMax : 0;
}

// ---- host: slice a tree description to a row range -------------------------

static uint64_t prefix_popcount(const uint64_t *w, uint64_t x) {  // set bits in [0, x)
    uint64_t r = 0;
    const uint64_t full = x >> 6;
    for (uint64_t i = 0; i < full; ++i) r += (uint64_t)__builtin_popcountll(w[i]);
    if (x & 63) r += (uint64_t)__builtin_popcountll(w[full] & ((1ull << (x & 63)) - 1));
    return r;
}

static void copy_bits(const uint64_t *w, uint64_t lo, uint64_t len, std::vector<uint64_t> &out) {
    const uint64_t nw = (len + 63) / 64;
    out.assign(nw, 0);
    const uint64_t sh = lo & 63, base = lo >> 6;
    const uint64_t src_words = (lo + len + 63) / 64;  // words of w that hold bits of the range
    for (uint64_t i = 0; i < nw; ++i) {
        uint64_t v = w[base + i] >> sh;
        if (sh && base + i + 1 < src_words) v |= w[base + i + 1] << (64 - sh);
        out[i] = v;
    }
    if (len & 63) out[nw - 1] &= (1ull << (len & 63)) - 1;
}

int slice_desc(const mbrwt_tree_desc &in, uint64_t a, uint64_t b, SlicedDesc &out) {
    const uint32_t N = in.num_nodes;
    out.sizes.assign(N, 0);
    out.words.assign(N, {});
    out.ptrs.assign(N, nullptr);
    std::vector<uint64_t> lo(N, 0), hi(N, 0);
    if (N) {
        lo[0] = a;
        hi[0] = b;
    }
    if (N && in.vec_size[0] != in.num_rows) {
        set_error("slice: the root's index column must hold num_rows bits");
        return MBRWT_ERR_INVALID;
    }
    for (uint32_t u = 0; u < N; ++u) {
        // the last shard ends every column: sizes must nest exactly
        const bool last = b == in.num_rows;
        if (hi[u] > in.vec_size[u] || lo[u] > hi[u] || (last && hi[u] != in.vec_size[u]) ||
            (hi[u] > lo[u] && !in.vec_words[u])) {
            set_error("slice: index column sizes do not nest (vec_size of a child != popcount of its parent)");
            return MBRWT_ERR_INVALID;
        }
        copy_bits(in.vec_words[u], lo[u], hi[u] - lo[u], out.words[u]);
        out.sizes[u] = hi[u] - lo[u];
        out.ptrs[u] = out.words[u].data();
        if (in.num_children[u]) {
            if (in.first_child[u] <= u || (uint64_t)in.first_child[u] + in.num_children[u] > N) {
                set_error("slice: children must follow their parent in BFS order");
                return MBRWT_ERR_INVALID;
            }
            const uint64_t clo = prefix_popcount(in.vec_words[u], lo[u]);
            const uint64_t chi = clo + prefix_popcount(out.words[u].data(), hi[u] - lo[u]);
            for (uint32_t c = 0; c < in.num_children[u]; ++c) {
                lo[in.first_child[u] + c] = clo;
                hi[in.first_child[u] + c] = chi;
            }
        }
    }
    out.desc = in;
    out.desc.num_rows = b - a;
    out.desc.vec_size = out.sizes.data();
    out.desc.vec_words = out.ptrs.data();
    return MBRWT_OK;
}

// ---- device: routing and reassembly ----------------------------------------

__global__ __launch_bounds__(256) void k_route(const uint64_t *__restrict__ rows, uint64_t n, uint64_t num_rows,
                                               uint64_t shard_rows, uint32_t *__restrict__ keys,
                                               uint32_t *__restrict__ iota, unsigned long long *err) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const uint64_t r = rows[i];
        bad |= r >= num_rows;
        keys[i] = r < num_rows ? (uint32_t)(r / shard_rows) : 0u;
        iota[i] = (uint32_t)i;
    }
    if (bad) atomicOr(err, 1ull);
}

// begin[k] = first sorted index of shard k (shards without rows keep
// UINT64_MAX, filled on the host); local[i] = the row inside its shard
__global__ __launch_bounds__(256) void k_route_finish(const uint64_t *__restrict__ rows,
                                                      const uint32_t *__restrict__ skeys,
                                                      const uint32_t *__restrict__ perm, uint64_t n,
                                                      uint64_t shard_rows, uint64_t *__restrict__ local,
                                                      uint64_t *__restrict__ begin) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const uint32_t k = skeys[i];
        local[i] = rows[perm[i]] - (uint64_t)k * shard_rows;
        if (i == 0 || skeys[i - 1] != k) begin[k] = i;
    }
}

__global__ __launch_bounds__(256) void k_gather_u64(const uint64_t *__restrict__ src, const uint32_t *__restrict__ perm,
                                                    uint64_t n, uint64_t *__restrict__ dst) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) dst[i] = src[perm[i]];
}

__global__ __launch_bounds__(256) void k_scatter_u8(const uint8_t *__restrict__ src, const uint32_t *__restrict__ perm,
                                                    uint64_t n, uint8_t *__restrict__ dst) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) dst[perm[i]] = src[i];
}

// a shard's row counts into the batch's order (cnt has n + 1 entries, the
// last one zero, and becomes the offsets by one exclusive scan)
__global__ __launch_bounds__(256) void k_scatter_counts(const uint32_t *__restrict__ perm,
                                                        const uint64_t *__restrict__ off, uint64_t n,
                                                        uint64_t *__restrict__ cnt) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs)
        cnt[perm[i]] = off[i + 1] - off[i];
}

// a shard's labels to their rows' places in the batch CSR (one lane per row;
// bound by the random 8-byte offset read and the random destination of each
// row: 0.14 ms per 2.7 M rows; 8 lanes per row measured no faster)
__global__ __launch_bounds__(256) void k_scatter_labels(const uint32_t *__restrict__ perm,
                                                        const uint64_t *__restrict__ off,
                                                        const uint32_t *__restrict__ src, uint64_t n,
                                                        const uint64_t *__restrict__ offsets,
                                                        uint32_t *__restrict__ cols) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const uint64_t b = off[i], e = off[i + 1];
        uint32_t *dst = cols + offsets[perm[i]];
        for (uint64_t k = b; k < e; ++k) dst[k - b] = src[k];
    }
}

__global__ __launch_bounds__(256) void k_add_u64(uint64_t *__restrict__ dst, const uint64_t *__restrict__ src,
                                                 uint64_t n, uint64_t add) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs)
        dst[i] += (src ? src[i] : 0) + add;
}

static unsigned grid_for(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 16384)); }

// The batch grouped by shard: perm (batch index of every sorted entry), local
// rows, and begin[0..K] on the host.
struct Routed {
    const uint32_t *perm = nullptr;
    const uint64_t *local = nullptr;
    std::vector<uint64_t> begin;
};

static int route(Ctx &c, const uint64_t *d_rows, uint64_t n, Routed &r, hipStream_t s) {
    const uint32_t K = (uint32_t)c.shards.size();
    if (n > 0x7FFFFFF0ull) {  // u32 batch indices, int item counts in hipCUB
        set_error("batch larger than 2^31 rows");
        return MBRWT_ERR_UNSUPPORTED;
    }
    int rc;
    // keys | sorted keys | iota | perm (u32 each)
    if ((rc = ensure(c.ws_sh_keys, 4 * n * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(c.ws_sh_local, (n + K + 1) * sizeof(uint64_t)))) return rc;
    uint32_t *keys = reinterpret_cast<uint32_t *>(c.ws_sh_keys.buf);
    uint32_t *skeys = keys + n, *iota = keys + 2 * n, *perm = keys + 3 * n;
    uint64_t *local = reinterpret_cast<uint64_t *>(c.ws_sh_local.buf);
    uint64_t *d_begin = local + n;
    int bits = 1;
    while (bits < 32 && (1ull << bits) < K) ++bits;
    size_t sort_bytes = 0;
    MBRWT_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, keys, skeys, iota, perm, (int)n, 0, bits, s));
    if ((rc = ensure(c.ws_sh_sort, sort_bytes))) return rc;
    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 8 * sizeof(uint64_t), s));
    hipLaunchKernelGGL(k_route, dim3(grid_for(n)), dim3(256), 0, s, d_rows, n, c.tree.num_rows, c.shard_rows, keys,
                       iota, reinterpret_cast<unsigned long long *>(c.d_scalars));
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipcub::DeviceRadixSort::SortPairs(c.ws_sh_sort.buf, sort_bytes, keys, skeys, iota, perm, (int)n, 0,
                                                 bits, s));
    MBRWT_HIP(hipMemsetAsync(d_begin, 0xFF, (K + 1) * sizeof(uint64_t), s));
    hipLaunchKernelGGL(k_route_finish, dim3(grid_for(n)), dim3(256), 0, s, d_rows, skeys, perm, n, c.shard_rows, local,
                       d_begin);
    MBRWT_HIP(hipGetLastError());
    r.begin.assign(K + 1, 0);
    MBRWT_HIP(hipMemcpyAsync(r.begin.data(), d_begin, (K + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, sizeof(uint64_t) * 4, hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (c.h_scalars[0] & 1) {
        set_error("row out of range");
        return MBRWT_ERR_RANGE;
    }
    r.begin[K] = n;
    for (uint32_t k = K; k-- > 0;)
        if (r.begin[k] == UINT64_MAX) r.begin[k] = r.begin[k + 1];
    r.perm = perm;
    r.local = local;
    return MBRWT_OK;
}

int sharded_get_rows(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets, uint32_t *d_cols, uint64_t cap,
                     uint64_t *needed, hipStream_t s) {
    if (n == 0) {
        MBRWT_HIP(hipMemsetAsync(d_offsets, 0, sizeof(uint64_t), s));
        MBRWT_HIP(hipStreamSynchronize(s));
        if (needed) *needed = 0;
        return MBRWT_OK;
    }
    if (n > 0x7FFFFFF0ull) {
        set_error("batch larger than 2^31 rows");
        return MBRWT_ERR_UNSUPPORTED;
    }
    Routed r;
    int rc;
    if ((rc = route(c, d_rows, n, r, s))) return rc;
    const uint32_t K = (uint32_t)c.shards.size();
    uint64_t total = 0;
    if (!d_cols || cap == 0) {
        // a sizing call: count the labels per shard (the V/L pass, no label
        // is materialised) instead of answering the whole query twice
        for (uint32_t k = 0; k < K; ++k) {
            const uint64_t b = r.begin[k], ns = r.begin[k + 1] - b;
            if (!ns) continue;
            uint64_t visits = 0, labels = 0;
            if ((rc = run_count_work(*c.shards[k], r.local + b, ns, &visits, &labels, s))) return rc;
            total += labels;
        }
        if (needed) *needed = total;
        if (total > 0) {
            set_error("cols_cap too small");
            return MBRWT_ERR_CAPACITY;
        }
    }
    // each shard answers its rows into its own workspaces (offsets in ws_rows,
    // labels in ws_out; the host-buffer API of a shard context is never used)
    total = 0;
    for (uint32_t k = 0; k < K; ++k) {
        const uint64_t b = r.begin[k], ns = r.begin[k + 1] - b;
        if (!ns) continue;
        Ctx &sc = *c.shards[k];
        if ((rc = ensure(sc.ws_rows, (ns + 1) * sizeof(uint64_t)))) return rc;
        if ((rc = ensure(sc.ws_out, 256 * sizeof(uint32_t)))) return rc;
        uint64_t need = 0;
        rc = run_get_rows(sc, r.local + b, ns, reinterpret_cast<uint64_t *>(sc.ws_rows.buf),
                          reinterpret_cast<uint32_t *>(sc.ws_out.buf), sc.ws_out.bytes / sizeof(uint32_t), &need, s);
        if (rc == MBRWT_ERR_CAPACITY) {
            if ((rc = ensure(sc.ws_out, (need + need / 4 + 64) * sizeof(uint32_t)))) return rc;
            rc = run_get_rows(sc, r.local + b, ns, reinterpret_cast<uint64_t *>(sc.ws_rows.buf),
                              reinterpret_cast<uint32_t *>(sc.ws_out.buf), sc.ws_out.bytes / sizeof(uint32_t), &need,
                              s);
        }
        if (rc) return rc;
        total += need;
    }
    if (needed) *needed = total;
    if (total > cap) {
        set_error("cols_cap too small");
        return MBRWT_ERR_CAPACITY;
    }
    if ((rc = ensure(c.ws_sh_cnt, (n + 1) * sizeof(uint64_t)))) return rc;
    uint64_t *cnt = reinterpret_cast<uint64_t *>(c.ws_sh_cnt.buf);
    MBRWT_HIP(hipMemsetAsync(cnt + n, 0, sizeof(uint64_t), s));
    for (uint32_t k = 0; k < K; ++k) {
        const uint64_t b = r.begin[k], ns = r.begin[k + 1] - b;
        if (!ns) continue;
        hipLaunchKernelGGL(k_scatter_counts, dim3(grid_for(ns)), dim3(256), 0, s, r.perm + b,
                           reinterpret_cast<const uint64_t *>(c.shards[k]->ws_rows.buf), ns, cnt);
        MBRWT_HIP(hipGetLastError());
    }
    size_t scan_bytes = 0;
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, cnt, d_offsets, n + 1, s));
    if ((rc = ensure(c.ws_sh_tmp, scan_bytes))) return rc;
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(c.ws_sh_tmp.buf, scan_bytes, cnt, d_offsets, n + 1, s));
    for (uint32_t k = 0; k < K; ++k) {
        const uint64_t b = r.begin[k], ns = r.begin[k + 1] - b;
        if (!ns) continue;
        const Ctx &sc = *c.shards[k];
        hipLaunchKernelGGL(k_scatter_labels, dim3(grid_for(ns)), dim3(256), 0, s, r.perm + b,
                           reinterpret_cast<const uint64_t *>(sc.ws_rows.buf),
                           reinterpret_cast<const uint32_t *>(sc.ws_out.buf), ns, d_offsets, d_cols);
        MBRWT_HIP(hipGetLastError());
    }
    return MBRWT_OK;
}

int sharded_get_batch(Ctx &c, const uint64_t *d_rows, const uint64_t *d_cols, uint64_t n, uint8_t *d_out,
                      hipStream_t s) {
    if (n == 0) return MBRWT_OK;
    if (n > 0x7FFFFFF0ull) {
        set_error("batch larger than 2^31 rows");
        return MBRWT_ERR_UNSUPPORTED;
    }
    Routed r;
    int rc;
    if ((rc = route(c, d_rows, n, r, s))) return rc;
    // sorted columns (u64) | shard answers (u8)
    if ((rc = ensure(c.ws_sh_cnt, n * sizeof(uint64_t) + n))) return rc;
    uint64_t *scols = reinterpret_cast<uint64_t *>(c.ws_sh_cnt.buf);
    uint8_t *sout = reinterpret_cast<uint8_t *>(scols + n);
    hipLaunchKernelGGL(k_gather_u64, dim3(grid_for(n)), dim3(256), 0, s, d_cols, r.perm, n, scols);
    MBRWT_HIP(hipGetLastError());
    for (uint32_t k = 0; k < c.shards.size(); ++k) {
        const uint64_t b = r.begin[k], ns = r.begin[k + 1] - b;
        if (!ns) continue;
        if ((rc = run_get_batch(*c.shards[k], r.local + b, scols + b, ns, sout + b, s))) return rc;
    }
    hipLaunchKernelGGL(k_scatter_u8, dim3(grid_for(n)), dim3(256), 0, s, sout, r.perm, n, d_out);
    MBRWT_HIP(hipGetLastError());
    return MBRWT_OK;
}

int sharded_count_labels(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_counts, hipStream_t s) {
    const uint64_t m = c.tree.num_columns;
    if (m) MBRWT_HIP(hipMemsetAsync(d_counts, 0, m * sizeof(uint64_t), s));
    if (n == 0) return MBRWT_OK;
    Routed r;
    int rc;
    if ((rc = route(c, d_rows, n, r, s))) return rc;
    if ((rc = ensure(c.ws_sh_cnt, std::max<uint64_t>(m, 1) * sizeof(uint64_t)))) return rc;
    uint64_t *tmp = reinterpret_cast<uint64_t *>(c.ws_sh_cnt.buf);
    for (uint32_t k = 0; k < c.shards.size(); ++k) {
        const uint64_t b = r.begin[k], ns = r.begin[k + 1] - b;
        if (!ns) continue;
        if ((rc = run_count_labels(*c.shards[k], r.local + b, ns, tmp, s))) return rc;
        hipLaunchKernelGGL(k_add_u64, dim3(grid_for(m)), dim3(256), 0, s, d_counts, tmp, m, 0ull);
        MBRWT_HIP(hipGetLastError());
    }
    return MBRWT_OK;
}

int sharded_count_work(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *visits, uint64_t *labels, hipStream_t s) {
    uint64_t v = 0, l = 0;
    if (n) {
        Routed r;
        int rc;
        if ((rc = route(c, d_rows, n, r, s))) return rc;
        for (uint32_t k = 0; k < c.shards.size(); ++k) {
            const uint64_t b = r.begin[k], ns = r.begin[k + 1] - b;
            if (!ns) continue;
            uint64_t vk = 0, lk = 0;
            if ((rc = run_count_work(*c.shards[k], r.local + b, ns, &vk, &lk, s))) return rc;
            v += vk;
            l += lk;
        }
    }
    if (visits) *visits = v;
    if (labels) *labels = l;
    return MBRWT_OK;
}

// BRWT::get_column over the whole matrix: the shards' ascending rows, shifted
// by the shards' first rows, concatenated in shard order
int sharded_get_column(Ctx &c, uint64_t column, uint64_t *d_rows, uint64_t rows_cap, uint64_t *rows_needed,
                       hipStream_t s) {
    if (column >= c.tree.num_columns) {
        set_error("column out of range");
        return MBRWT_ERR_RANGE;
    }
    uint64_t at = 0;
    bool short_cap = false;
    for (uint32_t k = 0; k < c.shards.size(); ++k) {
        uint64_t need = 0;
        const uint64_t room = (!short_cap && d_rows && rows_cap > at) ? rows_cap - at : 0;
        int rc = run_get_column(*c.shards[k], column, room ? d_rows + at : nullptr, room, &need, s);
        if (rc == MBRWT_ERR_CAPACITY) {
            short_cap = true;
        } else if (rc) {
            return rc;
        } else if (need && k) {
            hipLaunchKernelGGL(k_add_u64, dim3(grid_for(need)), dim3(256), 0, s, d_rows + at, nullptr, need,
                               (unsigned long long)k * c.shard_rows);
            MBRWT_HIP(hipGetLastError());
        }
        at += need;
    }
    if (rows_needed) *rows_needed = at;
    if (short_cap) {
        set_error("rows_cap too small");
        return MBRWT_ERR_CAPACITY;
    }
    return MBRWT_OK;
}

}  // namespace mbrwt

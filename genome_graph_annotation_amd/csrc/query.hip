// query.hip -- HIP kernels of the batched BRWT row query (gfx950 / CDNA4).
//
// Hot path: BRWT::get_row (BRWT.cpp:26-53) and the bit_vector_rrr<63>
// operator[] / rank1 it rides on (bit_vector.cpp:857-888), restated over the
// sibling-interleaved device image (mbrwt_internal.hpp).
//
// k_traverse: one lane per query row, depth-first over the tree in the
// reference's child order, with the pending frames of the descent in a
// register shift-stack (static register indices only, no scratch).  Lanes
// refill themselves with the next row of their grid-stride sequence as soon
// as their row finishes, so a wave stays full while rows of different
// lengths are in flight.  Every visit of an internal node at position j is
// ONE block read (64 B for arity 8) that yields the index bit and rank of all
// children at j; the rank of child c is rank_c(block) + popc(bits_c & below).
//
// Output: pass 1 writes each row's labels into a fixed slot of K labels and
// its count; an exclusive scan gives CSR offsets; a compaction copies slots
// to the CSR; rows with more than K labels are re-traversed straight into
// the CSR (pass 2 over the overflow list only).
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "mbrwt_internal.hpp"

namespace mbrwt {

enum { MODE_SLOTS = 0, MODE_DIRECT = 1, MODE_WORK = 2, MODE_COUNT = 3 };

struct TravParams {
    const DevNode *nodes;
    const uint64_t *rows;
    uint64_t n;                  // number of slots processed by this launch
    uint64_t num_rows;
    const uint32_t *slot_list;   // MODE_DIRECT: batch indices of the slots
    const uint32_t *order;       // optional: slot s processes batch index order[s]
    uint32_t K;
    uint32_t *temp;              // MODE_SLOTS: [n_batch][K]
    uint32_t *counts;            // MODE_SLOTS: [n_batch]
    uint32_t *ovf_list;          // MODE_SLOTS
    unsigned long long *scalars; // [0] total, [1] overflow count, [2] error flags, [3] visits, [4] labels
    const uint64_t *offsets;     // MODE_DIRECT
    uint32_t *cols;              // MODE_DIRECT
    unsigned long long *label_counts;  // MODE_COUNT: [num_columns]
};

template <typename MaskT>
__device__ __forceinline__ int ctz_m(MaskT m) {
    if constexpr (sizeof(MaskT) == 8) return __builtin_ctzll(m);
    else return __builtin_ctz(m);
}

template <int MAXD, typename MaskT>
struct Frames {
    uint32_t node[MAXD];
    uint32_t pos[MAXD];
    MaskT rem[MAXD];
    int sp;
    __device__ __forceinline__ void push(uint32_t v, uint32_t j, MaskT m) {
#pragma unroll
        for (int k = MAXD - 1; k > 0; --k) {
            node[k] = node[k - 1];
            pos[k] = pos[k - 1];
            rem[k] = rem[k - 1];
        }
        node[0] = v;
        pos[0] = j;
        rem[0] = m;
        ++sp;
    }
    __device__ __forceinline__ void pop() {
#pragma unroll
        for (int k = 0; k < MAXD - 1; ++k) {
            node[k] = node[k + 1];
            pos[k] = pos[k + 1];
            rem[k] = rem[k + 1];
        }
        --sp;
    }
};

// Per-lane sink for the labels of the current row.
template <int MODE>
struct Sink {
    uint32_t cnt;
    uint64_t slot_base;  // MODE_SLOTS: bi*K ; MODE_DIRECT: offsets[bi]
    uint64_t visits;
    __device__ __forceinline__ void emit(const TravParams &p, uint32_t label) {
        if constexpr (MODE == MODE_SLOTS) {
            if (cnt < p.K) p.temp[slot_base + cnt] = label;
        } else if constexpr (MODE == MODE_DIRECT) {
            p.cols[slot_base + cnt] = label;
        } else if constexpr (MODE == MODE_COUNT) {
            atomicAdd(&p.label_counts[label], 1ull);
        }
        ++cnt;
    }
};

template <typename MaskT>
__device__ __forceinline__ MaskT arity_mask(uint32_t a) {
    return a >= 8 * sizeof(MaskT) ? ~(MaskT)0 : (((MaskT)1 << a) - 1);
}

// Enter dnode v at position j of its children image (v's own index bit at
// this position is known to be set, or v is the super-root).
template <int MAXD, typename MaskT, int MODE>
__device__ __forceinline__ void enter(const TravParams &p, Frames<MAXD, MaskT> &st, Sink<MODE> &sk, uint32_t v,
                                      uint32_t j) {
    const DevNode *nd = p.nodes + v;
    const uint8_t kind = nd->kind;
    const uint32_t a = nd->arity;
    const uint8_t *base = reinterpret_cast<const uint8_t *>(nd->base);
    if constexpr (MODE == MODE_WORK) sk.visits += a;  // operator[] on every child (BRWT.cpp:30)
    if (kind == KIND_PLANE) {
        const uint8_t *blk = base + (uint64_t)(j >> 5) * nd->stride;
        const uint32_t t = j & 31;
        MaskT m = 0;
        for (uint32_t c = 0; c < a; c += 2) {
            const uint4 q = *reinterpret_cast<const uint4 *>(blk + 8u * c);
            m |= (MaskT)((q.y >> t) & 1u) << c;
            m |= (MaskT)((q.w >> t) & 1u) << (c + 1);
        }
        m &= arity_mask<MaskT>(a);
        if (m) {
            if (st.sp >= MAXD) {
                atomicOr(&p.scalars[2], 2ull);  // stack overflow: host picked MAXD too small
                return;
            }
            st.push(v, j, m);
        }
        return;
    }
    // all children are leaves: one mask per position
    uint64_t m;
    if (kind == KIND_MASK8) m = base[j];
    else if (kind == KIND_MASK16) m = reinterpret_cast<const uint16_t *>(base)[j];
    else if (kind == KIND_MASK32) m = reinterpret_cast<const uint32_t *>(base)[j];
    else m = reinterpret_cast<const uint64_t *>(base)[j];
    if (nd->flags & FLAG_CONSEC_LABELS) {
        const uint32_t l0 = nd->label;
        while (m) {
            sk.emit(p, l0 + (uint32_t)__builtin_ctzll(m));
            m &= m - 1;
        }
    } else {
        const uint32_t fc = nd->first_child;
        while (m) {
            sk.emit(p, p.nodes[fc + __builtin_ctzll(m)].label);
            m &= m - 1;
        }
    }
}

// One step: take the next set child of the top frame and descend into it.
template <int MAXD, typename MaskT, int MODE>
__device__ __forceinline__ void step(const TravParams &p, Frames<MAXD, MaskT> &st, Sink<MODE> &sk) {
    const uint32_t u = st.node[0];
    const uint32_t j = st.pos[0];
    MaskT m = st.rem[0];
    const int c = ctz_m(m);
    m &= m - 1;
    st.rem[0] = m;
    const DevNode *nu = p.nodes + u;
    const uint32_t v = nu->first_child + (uint32_t)c;
    const uint8_t *blk = reinterpret_cast<const uint8_t *>(nu->base) + (uint64_t)(j >> 5) * nu->stride + 8u * c;
    if (m == 0) st.pop();  // the frame has no children left: drop it before descending
    const DevNode *nv = p.nodes + v;
    if (nv->kind == KIND_LEAF) {
        sk.emit(p, nv->label);
        return;
    }
    const uint2 rb = *reinterpret_cast<const uint2 *>(blk);  // {rank before block, bits}
    const uint32_t below = (1u << (j & 31)) - 1u;
    const uint32_t jv = rb.x + (uint32_t)__builtin_popcount(rb.y & below);  // rank1(j) - 1
    enter<MAXD, MaskT, MODE>(p, st, sk, v, jv);
}

template <int MAXD, typename MaskT, int MODE>
__global__ __launch_bounds__(256) void k_traverse(TravParams p) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    Frames<MAXD, MaskT> st;
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        st.node[k] = 0;
        st.pos[k] = 0;
        st.rem[k] = 0;
    }
    st.sp = 0;
    Sink<MODE> sk;
    sk.cnt = 0;
    sk.visits = 0;
    sk.slot_base = 0;
    uint64_t bi = 0;
    unsigned long long acc_visits = 0, acc_labels = 0;

    auto begin_row = [&]() {
        bi = (MODE == MODE_DIRECT) ? (uint64_t)p.slot_list[s] : (p.order ? (uint64_t)p.order[s] : s);
        const uint64_t row = p.rows[bi];
        sk.cnt = 0;
        sk.visits = 0;
        if constexpr (MODE == MODE_SLOTS) sk.slot_base = bi * p.K;
        if constexpr (MODE == MODE_DIRECT) sk.slot_base = p.offsets[bi];
        if (row >= p.num_rows) {
            atomicOr(&p.scalars[2], 1ull);
            return;
        }
        enter<MAXD, MaskT, MODE>(p, st, sk, 0u, (uint32_t)row);
    };
    auto end_row = [&]() {
        if constexpr (MODE == MODE_SLOTS) {
            p.counts[bi] = sk.cnt;
            if (sk.cnt > p.K) {
                const unsigned long long k = atomicAdd(&p.scalars[1], 1ull);
                p.ovf_list[k] = (uint32_t)bi;
            }
        }
        if constexpr (MODE == MODE_WORK) {
            acc_visits += sk.visits;
            acc_labels += sk.cnt;
        }
    };

    bool active = s < p.n;
    if (active) begin_row();
    while (true) {
        if (active && st.sp == 0) {
            end_row();
            s += gstride;
            active = s < p.n;
            if (active) begin_row();
        }
        if (!__any(active)) break;
        if (active && st.sp > 0) step<MAXD, MaskT, MODE>(p, st, sk);
    }
    if constexpr (MODE == MODE_WORK) {
        if (acc_visits) atomicAdd(&p.scalars[3], acc_visits);
        if (acc_labels) atomicAdd(&p.scalars[4], acc_labels);
    }
}

// CSR compaction of the label slots (rows with <= K labels).
__global__ __launch_bounds__(256) void k_compact(const uint32_t *__restrict__ counts,
                                                 const uint64_t *__restrict__ offsets,
                                                 const uint32_t *__restrict__ temp, uint32_t K,
                                                 uint32_t *__restrict__ cols, uint64_t n) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        const uint32_t c = counts[i];
        if (c > K) continue;
        const uint64_t o = offsets[i];
        const uint32_t *src = temp + i * K;
        for (uint32_t k = 0; k < c; ++k) cols[o + k] = src[k];
    }
}

struct U32ToU64 {
    __host__ __device__ __forceinline__ uint64_t operator()(const uint32_t &x) const { return x; }
};

// Point queries: walk the column's root-to-leaf path (BRWT::get, BRWT.cpp:9-24).
__global__ __launch_bounds__(256) void k_get(const DevNode *__restrict__ nodes, const uint8_t *__restrict__ col_path,
                                             uint32_t path_len, const uint64_t *__restrict__ rows,
                                             const uint64_t *__restrict__ cols, uint64_t n, uint64_t num_rows,
                                             uint64_t num_cols, uint8_t *__restrict__ out,
                                             unsigned long long *scalars) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        const uint64_t row = rows[i], col = cols[i];
        if (row >= num_rows || col >= num_cols) {
            atomicOr(&scalars[2], 1ull);
            out[i] = 0;
            continue;
        }
        uint32_t v = 0, j = (uint32_t)row;
        uint8_t bit = 0;
        for (uint32_t k = 0; k < path_len; ++k) {
            const DevNode *nd = nodes + v;
            const uint32_t c = col_path[col * path_len + k];
            const uint8_t *base = reinterpret_cast<const uint8_t *>(nd->base);
            if (nd->kind == KIND_PLANE) {
                const uint2 rb = *reinterpret_cast<const uint2 *>(base + (uint64_t)(j >> 5) * nd->stride + 8u * c);
                const uint32_t t = j & 31;
                if (!((rb.y >> t) & 1u)) break;
                j = rb.x + (uint32_t)__builtin_popcount(rb.y & ((1u << t) - 1u));
                v = nd->first_child + c;
                if (nodes[v].kind == KIND_LEAF) {
                    bit = 1;
                    break;
                }
            } else {
                uint64_t m;
                if (nd->kind == KIND_MASK8) m = base[j];
                else if (nd->kind == KIND_MASK16) m = reinterpret_cast<const uint16_t *>(base)[j];
                else if (nd->kind == KIND_MASK32) m = reinterpret_cast<const uint32_t *>(base)[j];
                else m = reinterpret_cast<const uint64_t *>(base)[j];
                bit = (uint8_t)((m >> c) & 1u);
                break;
            }
        }
        out[i] = bit;
    }
}

// ------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------

namespace {

using TravFn = void (*)(TravParams);

template <int MODE>
TravFn pick_traverse(uint32_t depth, uint32_t max_arity) {
    const bool wide = max_arity > 32;
#define PICK(D)                                                               \
    if (depth <= D)                                                           \
        return wide ? (TravFn)k_traverse<D, uint64_t, MODE> : (TravFn)k_traverse<D, uint32_t, MODE>;
    PICK(4)
    PICK(8)
    PICK(16)
    PICK(32)
#undef PICK
    return nullptr;
}

int grid_for(Ctx &c, TravFn fn, uint64_t n) {
    int dev_cus = 0;
    (void)hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, c.device);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(fn), 256, 0) != hipSuccess ||
        per_cu <= 0)
        per_cu = 4;
    uint64_t resident = (uint64_t)std::max(1, dev_cus) * (uint64_t)per_cu;
    uint64_t need = (n + 255) / 256;
    return (int)std::max<uint64_t>(1, std::min(need, resident));
}

uint32_t auto_slots(const Ctx &c) {
    if (c.slot_labels) return c.slot_labels;
    const double mean = c.tree.num_rows ? (double)c.tree.num_relations / (double)c.tree.num_rows : 0.0;
    uint32_t k = 16;
    while (k < 4.0 * mean + 16.0 && k < 1024) k <<= 1;
    return k;
}

TravParams base_params(const Ctx &c) {
    TravParams p{};
    p.nodes = c.d_nodes;
    p.num_rows = c.tree.num_rows;
    p.scalars = reinterpret_cast<unsigned long long *>(c.d_scalars);
    return p;
}

}  // namespace

int ensure(Workspace &w, size_t bytes) {
    if (w.bytes >= bytes) return MBRWT_OK;
    if (w.buf) MBRWT_HIP(hipFree(w.buf));
    w.buf = nullptr;
    w.bytes = 0;
    size_t b = std::max<size_t>(bytes, 256);
    MBRWT_HIP(hipMalloc(&w.buf, b));
    w.bytes = b;
    return MBRWT_OK;
}

int run_get_rows(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets, uint32_t *d_cols, uint64_t cap,
                 uint64_t *needed, hipStream_t s) {
    if (n == 0) {
        MBRWT_HIP(hipMemsetAsync(d_offsets, 0, sizeof(uint64_t), s));
        MBRWT_HIP(hipStreamSynchronize(s));
        if (needed) *needed = 0;
        return MBRWT_OK;
    }
    if (c.tree.nodes.empty()) {  // BRWT(): every row is out of range
        set_error("query on an empty BRWT");
        return MBRWT_ERR_RANGE;
    }
    if (n > 0xFFFFFFFFull) {
        set_error("batch larger than 2^32 rows");
        return MBRWT_ERR_UNSUPPORTED;
    }
    const uint32_t K = auto_slots(c);
    TravFn fn = pick_traverse<MODE_SLOTS>(c.tree.stack_depth, c.tree.max_arity);
    TravFn fn_direct = pick_traverse<MODE_DIRECT>(c.tree.stack_depth, c.tree.max_arity);
    if (!fn || !fn_direct) {
        set_error("tree deeper than 32 levels of internal nodes");
        return MBRWT_ERR_UNSUPPORTED;
    }
    int rc;
    if ((rc = ensure(c.ws_temp, n * K * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(c.ws_counts, (n + 1) * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(c.ws_ovf, n * sizeof(uint32_t)))) return rc;
    size_t scan_bytes = 0;
    hipcub::TransformInputIterator<uint64_t, U32ToU64, const uint32_t *> it(
        reinterpret_cast<const uint32_t *>(c.ws_counts.buf), U32ToU64());
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, it, d_offsets, n + 1, s));
    if ((rc = ensure(c.ws_scan, scan_bytes))) return rc;

    TravParams p = base_params(c);
    p.rows = d_rows;
    p.n = n;
    p.K = K;
    p.temp = reinterpret_cast<uint32_t *>(c.ws_temp.buf);
    p.counts = reinterpret_cast<uint32_t *>(c.ws_counts.buf);
    p.ovf_list = reinterpret_cast<uint32_t *>(c.ws_ovf.buf);

    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 8 * sizeof(uint64_t), s));
    MBRWT_HIP(hipMemsetAsync(p.counts + n, 0, sizeof(uint32_t), s));
    const int grid = grid_for(c, fn, n);
    if (c.timing) MBRWT_HIP(hipEventRecord(c.ev0, s));
    hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, s, p);
    MBRWT_HIP(hipGetLastError());
    if (c.timing) MBRWT_HIP(hipEventRecord(c.ev1, s));
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(c.ws_scan.buf, scan_bytes, it, d_offsets, n + 1, s));
    MBRWT_HIP(hipMemcpyAsync(c.d_scalars, d_offsets + n, sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (c.timing) {
        float ms = 0;
        MBRWT_HIP(hipEventElapsedTime(&ms, c.ev0, c.ev1));
        c.timing_ms += ms;
        c.timing_launches += 1;
    }
    const uint64_t total = c.h_scalars[0], ovf = c.h_scalars[1], err = c.h_scalars[2];
    if (err & 1) {
        set_error("row out of range");
        return MBRWT_ERR_RANGE;
    }
    if (err & 2) {
        set_error("traversal stack overflow");
        return MBRWT_ERR_UNSUPPORTED;
    }
    if (needed) *needed = total;
    if (total > cap) {
        set_error("cols_cap too small");
        return MBRWT_ERR_CAPACITY;
    }
    {
        const uint64_t g = std::min<uint64_t>((n + 255) / 256, 8192);
        hipLaunchKernelGGL(k_compact, dim3((unsigned)g), dim3(256), 0, s, p.counts, d_offsets, p.temp, K, d_cols, n);
        MBRWT_HIP(hipGetLastError());
    }
    if (ovf) {
        TravParams q = p;
        q.n = ovf;
        q.slot_list = p.ovf_list;
        q.offsets = d_offsets;
        q.cols = d_cols;
        const int g2 = grid_for(c, fn_direct, ovf);
        hipLaunchKernelGGL(fn_direct, dim3(g2), dim3(256), 0, s, q);
        MBRWT_HIP(hipGetLastError());
    }
    return MBRWT_OK;
}

int run_count_work(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *visits, uint64_t *labels, hipStream_t s) {
    if (c.tree.nodes.empty()) return n ? MBRWT_ERR_RANGE : MBRWT_OK;
    TravFn fn = pick_traverse<MODE_WORK>(c.tree.stack_depth, c.tree.max_arity);
    if (!fn) return MBRWT_ERR_UNSUPPORTED;
    TravParams p = base_params(c);
    p.rows = d_rows;
    p.n = n;
    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 8 * sizeof(uint64_t), s));
    if (n) {
        hipLaunchKernelGGL(fn, dim3(grid_for(c, fn, n)), dim3(256), 0, s, p);
        MBRWT_HIP(hipGetLastError());
    }
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (c.h_scalars[2] & 1) return MBRWT_ERR_RANGE;
    if (c.h_scalars[2] & 2) return MBRWT_ERR_UNSUPPORTED;
    if (visits) *visits = c.h_scalars[3];
    if (labels) *labels = c.h_scalars[4];
    return MBRWT_OK;
}

int run_count_labels(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_counts, hipStream_t s) {
    if (c.tree.num_columns) MBRWT_HIP(hipMemsetAsync(d_counts, 0, c.tree.num_columns * sizeof(uint64_t), s));
    if (c.tree.nodes.empty()) return n ? MBRWT_ERR_RANGE : MBRWT_OK;
    TravFn fn = pick_traverse<MODE_COUNT>(c.tree.stack_depth, c.tree.max_arity);
    if (!fn) return MBRWT_ERR_UNSUPPORTED;
    TravParams p = base_params(c);
    p.rows = d_rows;
    p.n = n;
    p.label_counts = reinterpret_cast<unsigned long long *>(d_counts);
    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 8 * sizeof(uint64_t), s));
    if (n) {
        hipLaunchKernelGGL(fn, dim3(grid_for(c, fn, n)), dim3(256), 0, s, p);
        MBRWT_HIP(hipGetLastError());
    }
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (c.h_scalars[2] & 1) return MBRWT_ERR_RANGE;
    if (c.h_scalars[2] & 2) return MBRWT_ERR_UNSUPPORTED;
    return MBRWT_OK;
}

int run_get_batch(Ctx &c, const uint64_t *d_rows, const uint64_t *d_cols, uint64_t n, uint8_t *d_out, hipStream_t s) {
    if (n == 0) return MBRWT_OK;
    if (c.tree.nodes.empty()) return MBRWT_ERR_RANGE;
    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 8 * sizeof(uint64_t), s));
    const uint64_t g = std::min<uint64_t>((n + 255) / 256, 16384);
    hipLaunchKernelGGL(k_get, dim3((unsigned)g), dim3(256), 0, s, c.d_nodes, c.d_col_path, c.tree.path_len, d_rows,
                       d_cols, n, c.tree.num_rows, c.tree.num_columns, d_out,
                       reinterpret_cast<unsigned long long *>(c.d_scalars));
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (c.h_scalars[2] & 1) return MBRWT_ERR_RANGE;
    return MBRWT_OK;
}

}  // namespace mbrwt

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
#include <type_traits>

#include "device_access.hpp"
#include "mbrwt_internal.hpp"
#include "pack_block.hpp"

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
    uint32_t *chunk_counts;      // k_traverse_fast2: labels per 8-row chunk [n_batch / 8]
    uint32_t *ovf_list;          // MODE_SLOTS
    unsigned long long *scalars; // [0] total, [1] overflow count, [2] error flags, [3] visits, [4] labels
    const uint64_t *offsets;     // MODE_DIRECT
    uint32_t *cols;              // MODE_DIRECT
    unsigned long long *label_counts;  // MODE_COUNT: [num_columns]
    const CNode *cnodes;         // compact node records (group kernel)
    uint32_t n_lds;              // records [0, n_lds) are staged in LDS
    uint32_t folded;             // root folded into the super-root (V accounting)
    const uint32_t *label_map;   // pre-order index -> global column (Tree::label_perm; null = identity)
};

// MODE_DIRECT / MODE_COUNT write final columns; the slot modes keep pre-order
// indices and the compaction maps them
__device__ __forceinline__ uint32_t final_label(const uint32_t *map, uint32_t label) {
    return map ? gld(map + label) : label;
}

// The compaction kernels stage the label map in LDS when it is small (one
// random 4-byte global read per label measured 2.3 ms per 8 M labels on a
// greedy tree): `lds_entries` > 0 = the first kernel arguments' map copied
// into the dynamic LDS of the workgroup.
constexpr uint32_t kMapLdsMax = 16384;  // entries (64 KiB)
struct LabelMap {
    const uint32_t *g;
    const AS_LDS uint32_t *l;
    __device__ __forceinline__ uint32_t operator()(uint32_t x) const { return l ? l[x] : g ? gld(g + x) : x; }
};
__device__ __forceinline__ LabelMap stage_label_map(const uint32_t *map, uint32_t lds_entries) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_label_map[];
    if (!map || !lds_entries) return LabelMap{map, nullptr};
    for (uint32_t i = threadIdx.x; i < lds_entries; i += blockDim.x) lds_label_map[i] = gld(map + i);
    __syncthreads();
    return LabelMap{map, (const AS_LDS uint32_t *)lds_label_map};
}

// decoded node record
struct NodeInfo {
    uint64_t base;
    uint32_t first_child;
    uint32_t label;
    uint32_t stride;
    uint32_t arity;
    uint32_t kind;
    uint32_t flags;
};
__device__ __forceinline__ NodeInfo decode(uint64_t w0, uint64_t w1) {
    NodeInfo n;
    n.base = w0 & ((1ull << 48) - 1);
    n.kind = (uint32_t)(w0 >> 48) & 7u;
    n.flags = (uint32_t)(w0 >> 51) & 1u;
    if (n.kind == KIND_PACK && n.flags) n.kind = KIND_PACK2;  // CNode encoding (mbrwt_internal.hpp)
    n.stride = 1u << ((uint32_t)(w0 >> 52) & 15u);
    n.arity = (uint32_t)(w0 >> 56);
    n.first_child = (uint32_t)w1;
    n.label = (uint32_t)(w1 >> 32);
    return n;
}

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
            if (cnt < p.K) gst(p.temp + slot_base + cnt, label);
        } else if constexpr (MODE == MODE_DIRECT) {
            gst(p.cols + slot_base + cnt, final_label(p.label_map, label));
        } else if constexpr (MODE == MODE_COUNT) {
            atomicAdd(&p.label_counts[final_label(p.label_map, label)], 1ull);
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
    const DevNode nd = gld(p.nodes + v);
    const uint8_t kind = nd.kind;
    const uint32_t a = nd.arity;
    const uint64_t base = nd.base;
    if constexpr (MODE == MODE_WORK) sk.visits += a;  // operator[] on every child (BRWT.cpp:30)
    if (kind == KIND_PACKT) {  // the whole subtree below v at j, DFS pre-order
        Pack2Block pb;
        pb.load(base, j, nd.stride);
        const bool ok = packt_walk(
            p.nodes, v, [&](uint32_t o) { return pb.byte(o); }, pb.start(j % nd.stride),
            [&](uint32_t label) { sk.emit(p, label); },
            [&](uint32_t ar) {
                if constexpr (MODE == MODE_WORK) sk.visits += ar;
            });
        if (!ok) atomicOr(&p.scalars[2], 2ull);
        return;
    }
    if (kind == KIND_PACK2) {  // the whole subtree below v at j, in pre-order
        Pack2Block pb;
        pb.load(base, j, nd.stride);
        const uint32_t s = pb.start(j % nd.stride);
        const uint32_t m2 = pb.byte(s);
        uint32_t o1 = s + 1, o2 = s + 1 + (uint32_t)__builtin_popcount(m2);
        for (uint32_t A = 0; A < a; ++A) {
            if (!((m2 >> A) & 1u)) continue;
            const DevNode na = gld(p.nodes + nd.first_child + A);
            if constexpr (MODE == MODE_WORK) sk.visits += na.arity;
            for (uint32_t x = pb.byte(o1++); x; x &= x - 1) {
                const DevNode nb = gld(p.nodes + na.first_child + (uint32_t)__builtin_ctz(x));
                if constexpr (MODE == MODE_WORK) sk.visits += nb.arity;
                for (uint32_t m = pb.byte(o2++); m; m &= m - 1) sk.emit(p, nb.label + (uint32_t)__builtin_ctz(m));
            }
        }
        return;
    }
    if (kind == KIND_PACK) {  // children are MASK8 nodes: resolve them here, in child order
        PackBlock pb;
        pb.load(base, j);
        const uint32_t t = j % kPackSpan;
        uint32_t o = 0;
        for (uint32_t k = 0; k < a; ++k) {
            const uint32_t bk = pb.bits(k);
            if ((bk >> t) & 1u) {
                const DevNode ch = gld(p.nodes + nd.first_child + k);
                if constexpr (MODE == MODE_WORK) sk.visits += ch.arity;
                uint32_t m = pb.mask(o + (uint32_t)__builtin_popcount(bk & ((1u << t) - 1u)));
                while (m) {
                    sk.emit(p, ch.label + (uint32_t)__builtin_ctz(m));
                    m &= m - 1;
                }
            }
            o += (uint32_t)__builtin_popcount(bk);
        }
        return;
    }
    if (kind == KIND_PLANE) {
        const uint64_t blk = base + (uint64_t)(j >> 5) * nd.stride;
        const uint32_t t = j & 31;
        MaskT m = 0;
        for (uint32_t c = 0; c < a; c += 2) {
            const uint4 q = gld_at<uint4>(blk + 8u * c);
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
    if (kind == KIND_MASK8) m = gld_at<uint8_t>(base + j);
    else if (kind == KIND_MASK16) m = gld_at<uint16_t>(base + 2ull * j);
    else if (kind == KIND_MASK32) m = gld_at<uint32_t>(base + 4ull * j);
    else m = gld_at<uint64_t>(base + 8ull * j);
    if (nd.flags & FLAG_CONSEC_LABELS) {
        const uint32_t l0 = nd.label;
        while (m) {
            sk.emit(p, l0 + (uint32_t)__builtin_ctzll(m));
            m &= m - 1;
        }
    } else {
        const uint32_t fc = nd.first_child;
        while (m) {
            sk.emit(p, gld(p.nodes + fc + __builtin_ctzll(m)).label);
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
    const DevNode nu = gld(p.nodes + u);
    const uint32_t v = nu.first_child + (uint32_t)c;
    const uint64_t blk = nu.base + (uint64_t)(j >> 5) * nu.stride + 8u * c;
    if (m == 0) st.pop();  // the frame has no children left: drop it before descending
    const DevNode nv = gld(p.nodes + v);
    if (nv.kind == KIND_LEAF) {
        sk.emit(p, nv.label);
        return;
    }
    const uint2 rb = gld_at<uint2>(blk);  // {rank before block, bits}
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
        bi = (MODE == MODE_DIRECT) ? (uint64_t)gld(p.slot_list + s) : (p.order ? (uint64_t)gld(p.order + s) : s);
        const uint64_t row = gld(p.rows + bi);
        sk.cnt = 0;
        sk.visits = 0;
        if constexpr (MODE == MODE_SLOTS) sk.slot_base = bi * p.K;
        if constexpr (MODE == MODE_DIRECT) sk.slot_base = gld(p.offsets + bi);
        if (row >= p.num_rows) {
            atomicOr(&p.scalars[2], 1ull);
            return;
        }
        enter<MAXD, MaskT, MODE>(p, st, sk, 0u, (uint32_t)row);
        if constexpr (MODE == MODE_WORK) {
            // folded root: its own probe counts once, its children's only if its bit is set
            if (p.folded) sk.visits = sk.visits + 1 - ((st.sp == 0 && sk.cnt == 0) ? (uint64_t)gld(p.nodes).arity : 0ull);
        }
    };
    auto end_row = [&]() {
        if constexpr (MODE == MODE_SLOTS) {
            gst(p.counts + bi, sk.cnt);
            if (sk.cnt > p.K) {
                const unsigned long long k = atomicAdd(&p.scalars[1], 1ull);
                gst(p.ovf_list + k, (uint32_t)bi);
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

// ------------------------------------------------------------------------
// k_traverse_group: G lanes cooperate on one row (G = pow2ceil(max arity)).
// Visiting node u at position j, lane c of the group reads child c's
// {rank, bits} pair: the G 8-byte reads of one block are adjacent, so the
// memory pipeline sees ONE coalesced request per visit instead of one per
// lane-load (random requests, not bytes, bound this path: tools/
// gather_probe.hip).  Each stack level holds, per lane, the child index j_c
// of child c and, uniform in the group, the parent's first child and the
// mask of children still to visit.  Children are taken in order (DFS, the
// reference's output order); the index of the next child comes from lane
// c's register through a cross-lane shuffle.
// ------------------------------------------------------------------------
template <int MAXD, int CPL, typename MaskT>
struct GroupFrames {
    uint32_t jc[MAXD][CPL];  // per lane: position of child c*CPL+k in its own image
    uint32_t fc[MAXD];       // uniform: dnode of child 0
    MaskT pend[MAXD];        // uniform: children still to take (bit i = child i)
    int sp;
    __device__ __forceinline__ void push(const uint32_t (&j)[CPL], uint32_t f, MaskT p) {
#pragma unroll
        for (int k = MAXD - 1; k > 0; --k) {
#pragma unroll
            for (int q = 0; q < CPL; ++q) jc[k][q] = jc[k - 1][q];
            fc[k] = fc[k - 1];
            pend[k] = pend[k - 1];
        }
#pragma unroll
        for (int q = 0; q < CPL; ++q) jc[0][q] = j[q];
        fc[0] = f;
        pend[0] = p;
        ++sp;
    }
    __device__ __forceinline__ void pop() {
#pragma unroll
        for (int k = 0; k < MAXD - 1; ++k) {
#pragma unroll
            for (int q = 0; q < CPL; ++q) jc[k][q] = jc[k + 1][q];
            fc[k] = fc[k + 1];
            pend[k] = pend[k + 1];
        }
        --sp;
    }
};

// Per-group label sink: the labels of the current row are staged in LDS
// (kStageLabels per group) and written out once, contiguously, when the row
// ends.  Stores count in vmcnt on CDNA4, so a store issued inside the
// descent would hold up the wait of the next dependent block load; staging
// keeps the descent free of global stores.  Labels past the stage go
// straight to global memory (rare: rows with > kStageLabels labels).
constexpr uint32_t kStageLabels = 32;

template <int MODE>
struct GroupSink {
    uint32_t cnt;        // labels emitted so far (uniform)
    uint64_t slot_base;  // MODE_SLOTS: bi*K ; MODE_DIRECT: offsets[bi]
    uint64_t visits;
    AS_LDS uint32_t *stage;  // this group's LDS stage
    // lane-parallel emission: `label` goes to position cnt + rank
    __device__ __forceinline__ void put(const TravParams &p, uint32_t rank, uint32_t label) {
        const uint32_t pos = cnt + rank;
        if constexpr (MODE == MODE_DIRECT || MODE == MODE_COUNT) label = final_label(p.label_map, label);
        if constexpr (MODE == MODE_SLOTS || MODE == MODE_DIRECT) {
            if (pos < kStageLabels) {
                stage[pos] = label;
                return;
            }
        }
        if constexpr (MODE == MODE_SLOTS) {
            if (pos < p.K) gst(p.temp + slot_base + pos, label);
        } else if constexpr (MODE == MODE_DIRECT) {
            gst(p.cols + slot_base + pos, label);
        } else if constexpr (MODE == MODE_COUNT) {
            atomicAdd(&p.label_counts[label], 1ull);
        }
    }
    // end of row: the group's lanes copy the stage out, contiguously
    __device__ __forceinline__ void flush(const TravParams &p, uint32_t c, uint32_t G) {
        if constexpr (MODE == MODE_SLOTS || MODE == MODE_DIRECT) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint32_t lim = cnt < kStageLabels ? cnt : kStageLabels;
            if constexpr (MODE == MODE_SLOTS) lim = lim < p.K ? lim : p.K;
            for (uint32_t pos = c; pos < lim; pos += G) {
                if constexpr (MODE == MODE_SLOTS) gst(p.temp + slot_base + pos, (uint32_t)stage[pos]);
                else gst(p.cols + slot_base + pos, (uint32_t)stage[pos]);
            }
        }
    }
};

// spread the low G bits of x to every CPL-th bit position
template <int CPL>
__device__ __forceinline__ uint64_t spread_bits(uint64_t x, uint32_t G) {
    if constexpr (CPL == 1) return x;
    uint64_t r = 0;
    for (uint32_t i = 0; i < G; ++i) r |= ((x >> i) & 1ull) << (i * CPL);
    return r;
}

template <int MAXD, int CPL, typename MaskT, int MODE, bool NT = false>
__device__ __forceinline__ void group_visit(const TravParams &p, GroupFrames<MAXD, CPL, MaskT> &st, GroupSink<MODE> &sk,
                                            const NodeInfo &nd, uint32_t j, uint32_t c, uint32_t gbase,
                                            uint64_t gmask, uint32_t G) {
    const uint32_t a = nd.arity;
    const uint64_t base = nd.base;
    if constexpr (MODE == MODE_WORK) sk.visits += a;  // operator[] on every child (BRWT.cpp:30)
    if (nd.kind == KIND_PACK2) {
        // every lane walks the whole record; each emits the labels below its
        // own children at their rank among the node's labels (pre-order)
        Pack2Block pb;
        pb.load(base, j, nd.stride);
        const uint32_t s = pb.start(j % nd.stride);
        const uint32_t m2 = pb.byte(s);
        uint32_t o1 = s + 1, o2 = s + 1 + (uint32_t)__builtin_popcount(m2), total = 0;
        const uint64_t *cn = reinterpret_cast<const uint64_t *>(p.cnodes);
        for (uint32_t A = 0; A < a; ++A) {
            if (!((m2 >> A) & 1u)) continue;
            const uint32_t wa = nd.first_child + A;
            const NodeInfo na = decode(gld(cn + 2 * wa), gld(cn + 2 * wa + 1));
            if constexpr (MODE == MODE_WORK) sk.visits += na.arity;
            for (uint32_t x = pb.byte(o1++); x; x &= x - 1) {
                const uint32_t wb = na.first_child + (uint32_t)__builtin_ctz(x);
                const NodeInfo nb = decode(gld(cn + 2 * wb), gld(cn + 2 * wb + 1));
                if constexpr (MODE == MODE_WORK) sk.visits += nb.arity;
                const uint32_t lm = pb.byte(o2++);
                if (A / CPL == c) {
                    uint32_t r = total;
                    for (uint32_t mm = lm; mm; mm &= mm - 1) sk.put(p, r++, nb.label + (uint32_t)__builtin_ctz(mm));
                }
                total += (uint32_t)__builtin_popcount(lm);
            }
        }
        sk.cnt += total;
        return;
    }
    if (nd.kind == KIND_PACK) {
        // every lane holds the whole block; each emits the labels of its own
        // children at their rank among the node's labels (child order)
        PackBlock pb;
        pb.load(base, j);
        const uint32_t t = j % kPackSpan, below = (1u << t) - 1u;
        uint32_t o = 0, before = 0, total = 0;
        for (uint32_t k = 0; k < a; ++k) {
            const uint32_t bk = pb.bits(k);
            if ((bk >> t) & 1u) {
                const uint32_t m = pb.mask(o + (uint32_t)__builtin_popcount(bk & below));
                const NodeInfo ch = decode(gld(reinterpret_cast<const uint64_t *>(p.cnodes) + 2 * (nd.first_child + k)),
                                           gld(reinterpret_cast<const uint64_t *>(p.cnodes) + 2 * (nd.first_child + k) + 1));
                if constexpr (MODE == MODE_WORK) sk.visits += ch.arity;
                if (k / CPL == c) {
                    uint32_t mm = m, r = before;
                    for (; mm; mm &= mm - 1) sk.put(p, r++, ch.label + (uint32_t)__builtin_ctz(mm));
                }
                before += (uint32_t)__builtin_popcount(m);
                total += (uint32_t)__builtin_popcount(m);
            }
            o += (uint32_t)__builtin_popcount(bk);
        }
        sk.cnt += total;
        return;
    }
    if (nd.kind == KIND_PLANE) {
        const uint32_t t = j & 31;
        const uint32_t below = (1u << t) - 1u;
        uint32_t bit[CPL], jc[CPL];
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
            bit[q] = 0;
            jc[q] = 0;
        }
        if (c * CPL < a) {
            const uint64_t blk = base + (uint64_t)(j >> 5) * nd.stride + 8u * CPL * c;
            uint32_t rk[CPL], bw[CPL];
            if constexpr (CPL == 1) {
                const uint2 rb = gld_at_nt<uint2, NT>(blk);
                rk[0] = rb.x;
                bw[0] = rb.y;
            } else {
#pragma unroll
                for (int h = 0; h < CPL / 2; ++h) {
                    const uint4 q4 = gld_at_nt<uint4, NT>(blk + 16 * h);
                    rk[2 * h] = q4.x;
                    bw[2 * h] = q4.y;
                    rk[2 * h + 1] = q4.z;
                    bw[2 * h + 1] = q4.w;
                }
            }
#pragma unroll
            for (int q = 0; q < CPL; ++q) {
                if (c * CPL + q < a) {
                    bit[q] = (bw[q] >> t) & 1u;
                    jc[q] = rk[q] + (uint32_t)__builtin_popcount(bw[q] & below);  // rank1(j) - 1
                }
            }
        }
        uint64_t P = 0;
#pragma unroll
        for (int q = 0; q < CPL; ++q) P |= spread_bits<CPL>((__ballot(bit[q]) >> gbase) & gmask, G) << q;
        if (P) {
            if (st.sp >= MAXD) {
                if (c == 0) atomicOr(&p.scalars[2], 2ull);
                return;
            }
            st.push(jc, nd.first_child, (MaskT)P);
        }
        return;
    }
    uint64_t m;  // all children are leaves: one mask per position (uniform load)
    if (nd.kind == KIND_MASK8) m = gld_at_nt<uint8_t, NT>(base + j);
    else if (nd.kind == KIND_MASK16) m = gld_at<uint16_t>(base + 2ull * j);
    else if (nd.kind == KIND_MASK32) m = gld_at<uint32_t>(base + 4ull * j);
    else m = gld_at<uint64_t>(base + 8ull * j);
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
        const uint32_t cc = c * CPL + q;
        if (cc < a && ((m >> cc) & 1u)) {
            const uint32_t label =
                (nd.flags & FLAG_CONSEC_LABELS) ? nd.label + cc
                                                 : (uint32_t)(gld(reinterpret_cast<const uint64_t *>(p.cnodes) +
                                                                  2 * (nd.first_child + cc) + 1) >> 32);
            sk.put(p, (uint32_t)__builtin_popcountll(m & ((1ull << cc) - 1ull)), label);
        }
    }
    sk.cnt += (uint32_t)__builtin_popcountll(m);
}

template <int MAXD, int CPL, typename MaskT, int MODE, int WPE, bool NT = false>
__global__ __launch_bounds__(256, WPE) void k_traverse_group(TravParams p, uint32_t G) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c = lane & (G - 1);
    const uint32_t gbase = lane & ~(G - 1);
    const uint64_t gmask = G >= 64 ? ~0ull : ((1ull << G) - 1ull);
    const uint64_t groups_per_block = blockDim.x / G;
    const uint64_t gstride = (uint64_t)gridDim.x * groups_per_block;
    uint64_t s = (uint64_t)blockIdx.x * groups_per_block + threadIdx.x / G;

    GroupFrames<MAXD, CPL, MaskT> st;
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
#pragma unroll
        for (int q = 0; q < CPL; ++q) st.jc[k][q] = 0;
        st.fc[k] = 0;
        st.pend[k] = 0;
    }
    st.sp = 0;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_stage[];  // (256 / G) * kStageLabels
    // node records [0, n_lds) after the label stages
    AS_LDS uint64_t *lds_nodes = (AS_LDS uint64_t *)((AS_LDS uint32_t *)lds_stage + (blockDim.x / G) * kStageLabels);
    const uint64_t *gnodes = reinterpret_cast<const uint64_t *>(p.cnodes);
    for (uint32_t i = threadIdx.x; i < 2 * p.n_lds; i += blockDim.x) lds_nodes[i] = gld(gnodes + i);
    __syncthreads();
    auto node_info = [&](uint32_t w) -> NodeInfo {
        if (w < p.n_lds) return decode(lds_nodes[2 * w], lds_nodes[2 * w + 1]);
        return decode(gld(gnodes + 2 * w), gld(gnodes + 2 * w + 1));
    };
    GroupSink<MODE> sk;
    sk.cnt = 0;
    sk.visits = 0;
    sk.slot_base = 0;
    sk.stage = (AS_LDS uint32_t *)lds_stage + (threadIdx.x / G) * kStageLabels;
    uint64_t bi = 0;
    unsigned long long acc_visits = 0, acc_labels = 0;

    auto begin_row = [&]() {
        bi = (MODE == MODE_DIRECT) ? (uint64_t)gld(p.slot_list + s) : (p.order ? (uint64_t)gld(p.order + s) : s);
        const uint64_t row = gld(p.rows + bi);
        sk.cnt = 0;
        sk.visits = 0;
        if constexpr (MODE == MODE_SLOTS) sk.slot_base = bi * p.K;
        if constexpr (MODE == MODE_DIRECT) sk.slot_base = gld(p.offsets + bi);
        if (row >= p.num_rows) {
            if (c == 0) atomicOr(&p.scalars[2], 1ull);
            return;
        }
        const NodeInfo nd = node_info(0);
        group_visit<MAXD, CPL, MaskT, MODE, NT>(p, st, sk, nd, (uint32_t)row, c, gbase, gmask, G);
        if constexpr (MODE == MODE_WORK) {
            // folded root: its own probe counts once, its children's only if its bit is set
            if (p.folded) sk.visits = sk.visits + 1 - ((st.sp == 0 && sk.cnt == 0) ? (uint64_t)nd.arity : 0ull);
        }
    };
    auto end_row = [&]() {
        sk.flush(p, c, G);
        if constexpr (MODE == MODE_SLOTS) {
            if (c == 0) {
                gst(p.counts + bi, sk.cnt);
                if (sk.cnt > p.K) {
                    const unsigned long long k = atomicAdd(&p.scalars[1], 1ull);
                    gst(p.ovf_list + k, (uint32_t)bi);
                }
            }
        }
        if constexpr (MODE == MODE_WORK) {
            if (c == 0) {
                acc_visits += sk.visits;
                acc_labels += sk.cnt;
            }
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
        if (active && st.sp > 0) {
            MaskT P = st.pend[0];
            const uint32_t cs = (uint32_t)__builtin_ctzll((uint64_t)P);
            P &= P - 1;
            st.pend[0] = P;
            const uint32_t w = st.fc[0] + cs;
            uint32_t mine = st.jc[0][0];
#pragma unroll
            for (int q = 1; q < CPL; ++q)
                if ((cs % CPL) == (uint32_t)q) mine = st.jc[0][q];
            const uint32_t jw = (uint32_t)__shfl((int)mine, (int)(gbase + cs / CPL), 64);
            if (P == 0) st.pop();  // no children left at this level: drop it before descending
            const NodeInfo nd = node_info(w);
            if (nd.kind == KIND_LEAF) {
                if (c == 0) sk.put(p, 0, nd.label);
                sk.cnt += 1;
            } else {
                group_visit<MAXD, CPL, MaskT, MODE, NT>(p, st, sk, nd, jw, c, gbase, gmask, G);
            }
        }
    }
    if constexpr (MODE == MODE_WORK) {
        if (acc_visits) atomicAdd(&p.scalars[3], acc_visits);
        if (acc_labels) atomicAdd(&p.scalars[4], acc_labels);
    }
}

constexpr uint32_t kFastMaxd = 4;  // stack frames of k_traverse_fast2 (finalize_tree: fast_shape)

// Reductions over the 4 lanes of a group (lanes 4i..4i+3 = one DPP quad):
// quad_perm DPP moves, no LDS round trip.  All 4 lanes must be active.
__device__ __forceinline__ uint32_t quad_or(uint32_t v) {
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm(1,0,3,2)
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // quad_perm(2,3,0,1)
    return v;
}
// exclusive prefix sum of v over the quad (lane order); `total` = quad sum
__device__ __forceinline__ uint32_t quad_exclusive_sum(uint32_t v, uint32_t c, uint32_t &total) {
    uint32_t incl = v;
    uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x90, 0xF, 0xF, false);  // quad_perm(0,0,1,2)
    incl += c >= 1 ? y : 0u;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x40, 0xF, 0xF, false);  // quad_perm(0,0,0,1)
    incl += c >= 2 ? y : 0u;
    total = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0xFF, 0xF, 0xF, false);  // quad_perm(3,3,3,3)
    return incl - v;
}

// ------------------------------------------------------------------------
// k_traverse_fast2: the traversal kernel for the basic arity-<=8 trees
// (every internal node PLANE, MASK8 or PACK with arity <= 8, MASK8 labels
// consecutive, <= kFastMaxd stack frames, every non-leaf record in the LDS
// table -- Tree::fast_shape && lds_complete).  A group of 4 lanes answers a
// row (2 children per lane, 16 rows per wave).  Every iteration of the wave
// runs ONE inlined visit (a group starting a row visits the root in the same
// code as a group visiting a popped child): with 16 groups per wave at
// different places of their trees, every extra code path in the loop body
// is paid by the whole wave.  Visits:
//   PLANE -- one coalesced 64-byte block read (16 B per lane = {rank, bits}
//            of two children); child mask OR-reduced over the quad by DPP;
//            a stack frame (3 registers per lane) is pushed;
//   PACK  -- the same block read gives the children bits AND their MASK8
//            masks; the block is staged in LDS and each lane picks the masks
//            of its two children: a level costs no second dependent read;
//   PLANE with FLAG_MASK_CHILDREN (node kinds without MBRWT_KIND_PACK) -- block read, then
//            the (independent) mask reads of the set MASK8 children;
//   MASK8 -- leaf labels from one byte (only as the root's child).
// Labels are staged in LDS (32 per row) and flushed as 16-byte vectors when
// the row ends (vmcnt counts stores on CDNA4: no stores inside the descent).
// ------------------------------------------------------------------------
template <bool NT, bool SMALLK, bool P2>
__global__ __launch_bounds__(256, 8) void k_traverse_fast2(TravParams p) {
    // P2: trees with KIND_PACK2 nodes (one stack frame, no FLAG_MASK_CHILDREN
    // nodes): the PACK2 visit replaces the MASK_CHILDREN one, a shorter stack
    constexpr int kFastMaxd = P2 ? 1 : (int)mbrwt::kFastMaxd;
    constexpr uint64_t M48 = (1ull << 48) - 1;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c = lane & 3;
    const uint32_t gbase = lane & ~3u;
    const uint64_t gid = (uint64_t)blockIdx.x * 64 + threadIdx.x / 4;
    const uint64_t ngroups = (uint64_t)gridDim.x * 64;

    // LDS: 64 groups x kStageLabels labels | 64 groups x one 64-byte PACK block | node records
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_stage[];
    AS_LDS uint32_t *stage = (AS_LDS uint32_t *)lds_stage + (threadIdx.x / 4) * kStageLabels;
    AS_LDS uint32_t *pk = (AS_LDS uint32_t *)lds_stage + 64 * kStageLabels + (threadIdx.x / 4) * 16;
    AS_LDS uint64_t *lds_nodes = (AS_LDS uint64_t *)((AS_LDS uint32_t *)lds_stage + 64 * kStageLabels + 64 * 16);
    const uint64_t *gnodes = reinterpret_cast<const uint64_t *>(p.cnodes);
    for (uint32_t i = threadIdx.x; i < 2 * p.n_lds; i += blockDim.x) lds_nodes[i] = gld(gnodes + i);
    __syncthreads();

    uint32_t jc0[kFastMaxd], jc1[kFastMaxd], fp[kFastMaxd];  // fp = first_child << 8 | pending mask
#pragma unroll
    for (int k = 0; k < (int)kFastMaxd; ++k) jc0[k] = jc1[k] = fp[k] = 0;
    int sp = 0;
    uint32_t cnt = 0;
    // u32 chunk / slot indices: run_get_rows keeps batches below 2^31 rows
    uint32_t chunk = (uint32_t)gid;
    uint32_t ri = 0;
    uint32_t slot = chunk * 8;
    // output: the labels of a chunk's rows are packed back to back in the
    // chunk's 8*K-label region (rows with > K labels are left out for the
    // overflow pass), so the compaction is a contiguous copy per chunk
    uint32_t running = 0, chunk_total = 0;
    // the current row's first label in its chunk's region (recomputed, not held)
    auto slot_ptr = [&]() -> uint32_t * { return p.temp + (uint64_t)chunk * 8 * p.K + running; };

    // SMALLK: K == kStageLabels, every kept label fits the stage
    auto emit = [&](uint32_t pos, uint32_t label) {
        if (pos < kStageLabels) stage[pos] = label;
        else if (!SMALLK && pos < p.K) gst(slot_ptr() + pos, label);  // past the LDS stage
    };

    // rows: chunks of 8 consecutive slots per group, ids preloaded 2 per lane as
    // u32 (ids >= num_rows clamp to 0xFFFFFFFF >= num_rows)
    uint32_t r0 = 0, r1 = 0;
    auto clamp_row = [&](uint64_t r) -> uint32_t { return r < p.num_rows ? (uint32_t)r : 0xFFFFFFFFu; };
    auto load_chunk = [&]() {
        const uint64_t sb = (uint64_t)chunk * 8 + 2 * c;
        r0 = sb < p.n ? clamp_row(gld(p.rows + sb)) : 0u;
        r1 = sb + 1 < p.n ? clamp_row(gld(p.rows + sb + 1)) : 0u;
    };
    bool active = (uint64_t)slot < p.n, fresh = active;  // fresh: the slot's row has not been started
    if (active) load_chunk();

    while (true) {
        if (active && !fresh && sp == 0) {  // row done: flush its stage, count, next slot
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t lim = cnt < kStageLabels ? cnt : kStageLabels;
            uint32_t *const dst = slot_ptr();
            for (uint32_t q = c; q < lim; q += 4) gst(dst + q, (uint32_t)stage[q]);
            if (c == 0) {
                gst(p.counts + slot, cnt);
                if (cnt > p.K) {
                    const unsigned long long k = atomicAdd(&p.scalars[1], 1ull);
                    gst(p.ovf_list + k, slot);
                }
            }
            if (cnt <= p.K) running += cnt;
            chunk_total += cnt;
            if ((ri == 7 || slot + 1 == p.n) && c == 0) gst(p.chunk_counts + chunk, chunk_total);
            if (++ri == 8) {
                ri = 0;
                running = 0;
                chunk_total = 0;
                chunk += (uint32_t)ngroups;
                if ((uint64_t)chunk * 8 < p.n) load_chunk();
            }
            slot = chunk * 8 + ri;
            active = (uint64_t)chunk * 8 + ri < p.n;
            fresh = active;
        }
        if (!__any(active)) break;
        if (!active) continue;

        // the node to visit: the root for a fresh row, else the next pending child
        uint64_t w0, w1;
        uint32_t j;
        bool go = true;
        if (fresh) {
            fresh = false;
            cnt = 0;
            const uint32_t mine = (ri & 1) ? r1 : r0;
            j = (uint32_t)__shfl((int)mine, (int)(gbase + (ri >> 1)), 64);
            w0 = lds_nodes[0];
            w1 = lds_nodes[1];
            if ((uint64_t)j >= p.num_rows) {
                if (c == 0) atomicOr(&p.scalars[2], 1ull);
                go = false;
            }
        } else {
            uint32_t top = fp[0];
            const uint32_t cs = (uint32_t)__builtin_ctz(top & 0xFFu);
            top &= top - 1;
            fp[0] = top;
            const uint32_t w = (top >> 8) + cs;
            const uint32_t jsel = (cs & 1) ? jc1[0] : jc0[0];
            j = (uint32_t)__shfl((int)jsel, (int)(gbase + (cs >> 1)), 64);
            if ((top & 0xFFu) == 0) {
#pragma unroll
                for (int k = 0; k < (int)kFastMaxd - 1; ++k) {
                    jc0[k] = jc0[k + 1];
                    jc1[k] = jc1[k + 1];
                    fp[k] = fp[k + 1];
                }
                --sp;
            }
            w0 = lds_nodes[2 * w];
            w1 = lds_nodes[2 * w + 1];
        }
        if (!go) continue;

        const uint64_t base = w0 & M48;
        const uint32_t a = (uint32_t)(w0 >> 56);
        const uint32_t kind = (uint32_t)(w0 >> 48) & 7u;
        // the labels of this lane's two MASK8 children (masks m0, m1 with leaf
        // labels l0.., l1..) at their place among the node's labels
        auto emit_children = [&](uint32_t m0, uint32_t m1, uint32_t l0, uint32_t l1) {
            const uint32_t s0 = (uint32_t)__builtin_popcount(m0) + (uint32_t)__builtin_popcount(m1);
            uint32_t total;
            uint32_t pos = cnt + quad_exclusive_sum(s0, c, total);
            for (; m0; m0 &= m0 - 1) emit(pos++, l0 + (uint32_t)__builtin_ctz(m0));
            for (; m1; m1 &= m1 - 1) emit(pos++, l1 + (uint32_t)__builtin_ctz(m1));
            cnt += total;
        };
        if (P2 && ((w0 >> 48) & 15u) == 15u) {  // KIND_PACK2 (kind PACK + flag): the subtree below at j
            // one coalesced 64-byte block read; staged in LDS, each lane takes
            // children 2c, 2c+1 of the node: their m1 bytes, then the leaf
            // masks of their set children (offsets by quad scans)
            const uint32_t lgs = (uint32_t)(w0 >> 52) & 15u;  // log2(span)
            const uint32_t t = j & ((1u << lgs) - 1u);
            const uint4 q = gld_at_nt<uint4, NT>(base + (uint64_t)(j >> lgs) * kPack2Block + 16u * c);
            ((AS_LDS u32x4_t *)pk)[c] = u32x4_t{q.x, q.y, q.z, q.w};
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const AS_LDS uint8_t *pb = (const AS_LDS uint8_t *)pk;
            uint32_t s = pb[t];
            if (pb[0] == 0) {
                // rare (spilled block): the position's record is copied into the
                // group's LDS slot -- list = u16 start[S+1], then the records;
                // builders keep every record <= 64 bytes (mbrwt_internal.hpp)
                const uint64_t la = ((uint64_t)pk[3] << 32) | pk[2];
                const uint32_t s0 = gld_at<uint16_t>(la + 2ull * t), len = gld_at<uint16_t>(la + 2ull * t + 2) - s0;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();  // every lane has read the list address
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                AS_LDS uint8_t *pw = (AS_LDS uint8_t *)pk;
                for (uint32_t o = c; o < len; o += 4) pw[o] = gld_at<uint8_t>(la + s0 + o);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                s = 0;
            }
            const uint32_t fc = (uint32_t)w1;
            // the record walk: lane c takes children 2c, 2c+1 of the node
            auto walk = [&](auto rd) {
                const uint32_t m2 = rd(s);
                const uint32_t A0 = 2 * c;
                const uint32_t bA0 = (m2 >> A0) & 1u, bA1 = (m2 >> (A0 + 1)) & 1u;
                const uint32_t i0 = s + 1 + (uint32_t)__builtin_popcount(m2 & ((1u << A0) - 1u));
                const uint32_t m10 = bA0 ? rd(i0) : 0u;
                const uint32_t m11 = bA1 ? rd(i0 + bA0) : 0u;
                const uint32_t n1 = (uint32_t)__builtin_popcount(m10) + (uint32_t)__builtin_popcount(m11);
                uint32_t n1_tot;
                const uint32_t o2 = s + 1 + (uint32_t)__builtin_popcount(m2) + quad_exclusive_sum(n1, c, n1_tot);
                uint32_t nl = 0;
#pragma nounroll
                for (uint32_t k = 0; k < n1; ++k) nl += (uint32_t)__builtin_popcount(rd(o2 + k));
                uint32_t ltot;
                uint32_t pos = cnt + quad_exclusive_sum(nl, c, ltot);
                uint32_t o = o2;
#pragma unroll
                for (uint32_t h = 0; h < 2; ++h) {
                    uint32_t x = h ? m11 : m10;
                    if (!x) continue;
                    const uint32_t fa = (uint32_t)lds_nodes[2 * (fc + A0 + h) + 1];  // first MASK8 child of A
                    for (; x; x &= x - 1) {
                        const uint32_t l = (uint32_t)(lds_nodes[2 * (fa + (uint32_t)__builtin_ctz(x)) + 1] >> 32);
                        for (uint32_t lm = rd(o++); lm; lm &= lm - 1) emit(pos++, l + (uint32_t)__builtin_ctz(lm));
                    }
                }
                return ltot;
            };
            const uint32_t ltot = walk([&](uint32_t o) -> uint32_t { return pb[o]; });
            cnt += ltot;
            continue;
        }
        if (kind == KIND_PACK) {
            const uint32_t t = j % kPackSpan, below = (1u << t) - 1u;
            const uint4 q = gld_at_nt<uint4, NT>(base + (uint64_t)(j / kPackSpan) * kPackBlock + 16u * c);
            const uint32_t lo = q.x & 0xFFFFu, hi = q.x >> 16;  // bits of children 2c, 2c+1
            const uint32_t b0 = (lo >> t) & 1u, b1 = (hi >> t) & 1u;
            uint32_t pairs;
            const uint32_t pre = quad_exclusive_sum((uint32_t)__builtin_popcount(q.x), c, pairs);
            ((AS_LDS u32x4_t *)pk)[c] = u32x4_t{q.x, q.y, q.z, q.w};
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t o0 = pre + (uint32_t)__builtin_popcount(lo & below);
            const uint32_t o1 = pre + (uint32_t)__builtin_popcount(lo) + (uint32_t)__builtin_popcount(hi & below);
            uint32_t m0 = 0, m1 = 0, l0 = 0, l1 = 0;
            const uint32_t fc = (uint32_t)w1;
            if (pairs <= kPackArea) {
                const AS_LDS uint8_t *pb = (const AS_LDS uint8_t *)pk;
                if (b0) m0 = pb[pack_area_byte(o0)];
                if (b1) m1 = pb[pack_area_byte(o1)];
            } else {  // spilled block: area bytes 0..7 hold the list's address
                const uint64_t sa = ((uint64_t)pk[2] << 32) | pk[1];
                if (b0) m0 = gld_at_nt<uint8_t, NT>(sa + o0);
                if (b1) m1 = gld_at_nt<uint8_t, NT>(sa + o1);
            }
            if (b0) l0 = (uint32_t)(lds_nodes[2 * (fc + 2 * c) + 1] >> 32);
            if (b1) l1 = (uint32_t)(lds_nodes[2 * (fc + 2 * c + 1) + 1] >> 32);
            emit_children(m0, m1, l0, l1);
            continue;
        }
        if (kind == KIND_MASK8) {  // leaves below: labels from the mask
            const uint32_t m = gld_at_nt<uint8_t, NT>(base + j);
            const uint32_t l0 = (uint32_t)(w1 >> 32);
#pragma unroll
            for (uint32_t q = 0; q < 2; ++q) {
                const uint32_t cc = 2 * c + q;
                if ((m >> cc) & 1u) emit(cnt + (uint32_t)__builtin_popcount(m & ((1u << cc) - 1u)), l0 + cc);
            }
            cnt += (uint32_t)__builtin_popcount(m);
            continue;
        }
        // KIND_PLANE: one coalesced 64-byte block read, 2 children per lane
        const uint32_t stride = 1u << ((uint32_t)(w0 >> 52) & 15u);
        const uint32_t t = j & 31, below = (1u << t) - 1u;
        uint32_t b0 = 0, b1 = 0, j0 = 0, j1 = 0;
        if (2 * c < a) {
            const uint4 q = gld_at_nt<uint4, NT>(base + (uint64_t)(j >> 5) * stride + 16u * c);
            b0 = (q.y >> t) & 1u;
            b1 = (2 * c + 1 < a) ? (q.w >> t) & 1u : 0u;
            j0 = q.x + (uint32_t)__builtin_popcount(q.y & below);
            j1 = q.z + (uint32_t)__builtin_popcount(q.w & below);
        }
        const uint32_t fc = (uint32_t)w1;
        if (!P2 && ((w0 >> 51) & 1u)) {  // FLAG_MASK_CHILDREN: the set children's mask reads, together
            uint32_t m0 = 0, m1 = 0, l0 = 0, l1 = 0;
            if (b0) {
                const uint32_t w = fc + 2 * c;
                m0 = gld_at_nt<uint8_t, NT>((lds_nodes[2 * w] & M48) + j0);
                l0 = (uint32_t)(lds_nodes[2 * w + 1] >> 32);
            }
            if (b1) {
                const uint32_t w = fc + 2 * c + 1;
                m1 = gld_at_nt<uint8_t, NT>((lds_nodes[2 * w] & M48) + j1);
                l1 = (uint32_t)(lds_nodes[2 * w + 1] >> 32);
            }
            emit_children(m0, m1, l0, l1);
            continue;
        }
        const uint32_t P = quad_or((b0 | (b1 << 1)) << (2 * c));  // child k <- bit k
        if (P) {
            if (sp >= (int)kFastMaxd) {
                if (c == 0) atomicOr(&p.scalars[2], 2ull);
                continue;
            }
#pragma unroll
            for (int k = kFastMaxd - 1; k > 0; --k) {
                jc0[k] = jc0[k - 1];
                jc1[k] = jc1[k - 1];
                fp[k] = fp[k - 1];
            }
            jc0[0] = j0;
            jc1[0] = j1;
            fp[0] = (fc << 8) | P;
            ++sp;
        }
    }
}

// ------------------------------------------------------------------------
// k_traverse_p2w: the traversal kernel for trees whose super-root's children
// are all KIND_PACK2 nodes (the basic arity-8 trees at the Kingsford and
// RefSeq shapes).  A wave resolves a ROWBLOCK of 16 consecutive query rows in
// wave-uniform phases, so every iteration runs ONE code path for all 16 of
// its 4-lane groups (k_traverse_fast2 runs the row flush, the root visit and
// the PACK2 visit in nearly every iteration, for groups at different places):
//   root phase -- group g reads the super-root's 64-byte block at its row
//                 (BRWT.cpp:30 + :43 for every child of the root at once);
//                 its child mask P_g and the children's positions j_k;
//   items      -- the set (row, child) pairs of the rowblock, numbered in
//                 (row, child) order = the reference's output order
//                 (BRWT.cpp:45-51), listed in LDS (prefix of popc(P_g) over
//                 the groups by 4 ballots);
//   rounds     -- group g resolves item 16r + g: ONE 64-byte PACK2 block read
//                 (the child's whole 3-level subtree at j_k), the record walk
//                 counts the item's labels (quad scans), a wave scan over the
//                 round's items places them after all earlier items, and the
//                 labels go to the wave's LDS ring;
//   flush      -- complete 64-label units of the ring are stored as 256-byte
//                 wave-wide stores into the rowblock's temp region (full
//                 lines: no partial-line write amplification), the rest at
//                 the rowblock's end.
// Row counts come from the items' label positions; a rowblock with more than
// C labels stores none and lists its rows for the direct pass.
// ------------------------------------------------------------------------
constexpr uint32_t kP2wItems = 128;                      // <= 16 rows x 8 children
constexpr uint32_t kP2wWaveWords = kP2wItems + 32 + 132 + 20 + 16 * 16;  // + ring: items j | k | ipos | gfirst | blocks

struct P2wParams {
    const uint64_t *rows;
    uint64_t n;
    uint64_t num_rows;
    uint64_t root_base;       // dnode 0's PLANE image
    uint32_t root_stride;     // its bytes per 32-position block
    uint32_t table_words;     // Tree::p2w_table
    const uint32_t *table;
    uint32_t C;               // label capacity of a rowblock's temp region
    uint32_t S;               // LDS ring labels per wave (power of two >= 128)
    uint32_t *temp;           // [n_blocks][C]
    uint32_t *counts;         // [n] labels per row
    uint32_t *block_counts;   // [n_blocks] labels per rowblock
    uint32_t *ovf_list;       // rows of overflowing rowblocks
    unsigned long long *scalars;  // [1] overflow rows, [2] error flags
};

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// (A register prefetch of a group's next block measured +1 % at 8 waves per
// SIMD and -7 % at 6: removed)
template <bool NT, typename LT = uint32_t>
__global__ __launch_bounds__(256, 8) void k_traverse_p2w(P2wParams p) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_p2w[];
    const uint32_t lane = threadIdx.x & 63, c = lane & 3, g = lane >> 2, gb = lane & ~3u;
    // wave-uniform values are made scalar (SGPRs): VGPRs are the occupancy limit
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t i = threadIdx.x; i < p.table_words; i += blockDim.x) lds_p2w[i] = gld(p.table + i);
    __syncthreads();
    const AS_LDS uint32_t *tab = (const AS_LDS uint32_t *)lds_p2w;
    const uint32_t R = __builtin_amdgcn_readfirstlane(tab[0]), nA = __builtin_amdgcn_readfirstlane(tab[1]);
    const AS_LDS uint32_t *roots = tab + 4;
    const AS_LDS uint32_t *afc = roots + 4 * R;
    const AS_LDS uint32_t *blab = afc + nA;
    AS_LDS uint32_t *wbase = (AS_LDS uint32_t *)lds_p2w + ((p.table_words + 3) & ~3u) + wv * (kP2wWaveWords + p.S);
    AS_LDS uint32_t *items_j = wbase;                                 // [128] item position j
    AS_LDS uint8_t *items_k = (AS_LDS uint8_t *)(wbase + kP2wItems);  // [128] item child k
    AS_LDS uint32_t *ipos = wbase + kP2wItems + 32;                   // [129] item's first label; [T] = total
    AS_LDS uint32_t *gfirst = ipos + 132;                             // [17] group's first item; [16] = T
    AS_LDS uint32_t *pk = gfirst + 20 + 16 * g;                       // the group's staged 64-byte block
    AS_LDS uint32_t *ring = gfirst + 20 + 256;                        // S labels
    const AS_LDS uint8_t *pb = (const AS_LDS uint8_t *)pk;
    const uint32_t smask = p.S - 1;
    constexpr uint32_t kNone = 0xFFFFFFFFu;  // no row (ids are < num_rows <= 2^32 - 1)

    const uint64_t nblocks = (p.n + 15) / 16;
    const uint64_t wstride = (uint64_t)gridDim.x * 4;
    // the row of group g in rowblock b (out-of-range ids raise the error flag)
    auto load_row = [&](uint64_t b) -> uint32_t {
        const uint64_t r0 = b * 16;
        if (b >= nblocks || r0 + g >= p.n) return kNone;
        const uint64_t r = gld(p.rows + r0 + g);
        if (r < p.num_rows) return (uint32_t)r;
        if (c == 0) atomicOr(&p.scalars[2], 1ull);
        return kNone;
    };
    // the super-root's 64-byte block at `row` (16 bytes per lane: {rank, bits} of children 2c, 2c+1)
    auto root_load = [&](uint32_t row) -> uint4 {
        uint4 q = make_uint4(0, 0, 0, 0);
        if (row != kNone && 2 * c < R)
            q = gld_at_nt<uint4, NT>(p.root_base + (uint64_t)(row >> 5) * p.root_stride + 16u * c);
        return q;
    };
    // the PACK2 block of item i (the child's whole 3-level subtree at j)
    auto item_load = [&](uint32_t i, uint32_t T) -> uint4 {
        uint4 q = make_uint4(0, 0, 0, 0);
        if (i < T) {
            const uint32_t j = items_j[i], k = items_k[i];
            const uint64_t ubase = (uint64_t)roots[4 * k] | ((uint64_t)roots[4 * k + 1] << 32);
            q = gld_at_nt<uint4, NT>(ubase + (uint64_t)(j >> roots[4 * k + 2]) * kPack2Block + 16u * c);
        }
        return q;
    };

    uint64_t rb = (uint64_t)blockIdx.x * 4 + wv;
    for (; rb < nblocks; rb += wstride) {
        const uint64_t r0 = rb * 16;
        const uint32_t nr = (uint32_t)(p.n - r0 < 16 ? p.n - r0 : 16);
        // LT: the temp region's label type (u16 when every label is < 2^16:
        // half the traversal's writes and the compaction's reads)
        LT *const out = reinterpret_cast<LT *>(p.temp) + rb * (uint64_t)p.C;

        // ---- root phase: the super-root's block at group g's row ----
        const uint32_t row = load_row(rb);
        const uint4 qr = root_load(row);
        uint32_t P = 0, j0 = 0, j1 = 0;
        if (row != kNone && 2 * c < R) {
            const uint32_t t = row & 31, below = (1u << t) - 1u;
            const uint32_t b0 = (qr.y >> t) & 1u, b1 = (2 * c + 1 < R) ? (qr.w >> t) & 1u : 0u;
            j0 = qr.x + (uint32_t)__builtin_popcount(qr.y & below);
            j1 = qr.z + (uint32_t)__builtin_popcount(qr.w & below);
            P = (b0 | (b1 << 1)) << (2 * c);
        }
        P = quad_or(P);
        // ---- items in (row, child) order ----
        {
            const uint32_t ng = (uint32_t)__builtin_popcount(P);
            uint32_t pre = 0;
#pragma unroll
            for (uint32_t b = 0; b < 4; ++b) {
                const uint64_t M = __ballot(c == 0 && ((ng >> b) & 1u));
                pre += (uint32_t)__popcll(M & ((1ull << gb) - 1ull)) << b;
            }
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
                const uint32_t k = 2 * c + h;
                if ((P >> k) & 1u) {
                    const uint32_t idx = pre + (uint32_t)__builtin_popcount(P & ((1u << k) - 1u));
                    items_j[idx] = h ? j1 : j0;
                    items_k[idx] = (uint8_t)k;
                }
            }
            if (c == 0) gfirst[g] = pre;
            if (lane == 60) gfirst[16] = pre + ng;
        }
        wave_sync_lds();
        const uint32_t T = __builtin_amdgcn_readfirstlane(gfirst[16]);

        // ---- rounds: group g resolves item ib + g ----
        uint32_t running = 0, flushed = 0;  // wave-uniform label positions in the rowblock
        for (uint32_t ib = 0; ib < T; ib += 16) {
            const uint32_t i = ib + g;
            const bool act = i < T;
            const uint4 q = item_load(i, T);
            uint32_t j = 0, k = 0;
            if (act) {
                j = items_j[i];
                k = items_k[i];
            }
            const uint32_t lgs = roots[4 * k + 2], aidx = roots[4 * k + 3];
            const uint32_t t = j & ((1u << lgs) - 1u);
            if (act) ((AS_LDS u32x4_t *)pk)[c] = u32x4_t{q.x, q.y, q.z, q.w};
            wave_sync_lds();
            uint32_t s = act ? pb[t] : 0u;
            if (act && pb[0] == 0) {
                // spilled block: copy the position's record into the group's
                // slot (list = u16 start[S+1], then the records; <= 64 bytes)
                const uint64_t la = ((uint64_t)pk[3] << 32) | pk[2];
                const uint32_t s0 = gld_at<uint16_t>(la + 2ull * t), len = gld_at<uint16_t>(la + 2ull * t + 2) - s0;
                wave_sync_lds();  // every lane has read the list address
                AS_LDS uint8_t *pw = (AS_LDS uint8_t *)pk;
                for (uint32_t o = c; o < len; o += 4) pw[o] = gld_at<uint8_t>(la + s0 + o);
                wave_sync_lds();
                s = 0;
            }
            // record walk, part 1: this lane's children A = 2c, 2c+1 of the
            // PACK2 node, their m1 bytes, the count of their labels
            const uint32_t m2 = act ? pb[s] : 0u;
            const uint32_t A0 = 2 * c;
            const uint32_t bA0 = (m2 >> A0) & 1u, bA1 = (m2 >> (A0 + 1)) & 1u;
            const uint32_t i0 = s + 1 + (uint32_t)__builtin_popcount(m2 & ((1u << A0) - 1u));
            const uint32_t m10 = bA0 ? pb[i0] : 0u;
            const uint32_t m11 = bA1 ? pb[i0 + bA0] : 0u;
            const uint32_t n1 = (uint32_t)__builtin_popcount(m10) + (uint32_t)__builtin_popcount(m11);
            uint32_t n1_tot;
            const uint32_t o2 = s + 1 + (uint32_t)__builtin_popcount(m2) + quad_exclusive_sum(n1, c, n1_tot);
            uint32_t nl = 0;
#pragma nounroll
            for (uint32_t e = 0; e < n1; ++e) nl += (uint32_t)__builtin_popcount(pb[o2 + e]);
            uint32_t ltot;
            const uint32_t lofs = quad_exclusive_sum(nl, c, ltot);
            // the item's first label: a wave scan of the items' totals (lanes of
            // a group hold the same total; groups are in item order)
            uint32_t x = ltot;
#pragma unroll
            for (uint32_t d = 4; d < 64; d <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
                if (lane >= d) x += y;
            }
            const uint32_t rtot = __builtin_amdgcn_readlane(x, 63);
            const uint32_t ibase = running + x - ltot;
            if (act && c == 0) ipos[i] = ibase;
            // a round that does not fit the ring (rare): pending ring labels
            // first, then this round's labels straight to the temp region
            const bool direct = rtot + (running - flushed) > p.S;
            if (direct) {
                for (uint32_t q2 = flushed + lane; q2 < running; q2 += 64)
                    if (q2 < p.C) gst(out + q2, (LT)ring[q2 & smask]);
                wave_sync_lds();
            }
            // part 2: the labels, in the record's (pre-)order
            uint32_t pos = ibase + lofs;
            uint32_t o = o2;
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
                uint32_t xm = h ? m11 : m10;
                if (!xm) continue;
                const uint32_t fb = afc[aidx + A0 + h];  // first B of this A (index into blab)
                for (; xm; xm &= xm - 1) {
                    const uint32_t l = blab[fb + (uint32_t)__builtin_ctz(xm)];
                    for (uint32_t lm = pb[o++]; lm; lm &= lm - 1, ++pos) {
                        const uint32_t label = l + (uint32_t)__builtin_ctz(lm);
                        if (!direct) ring[pos & smask] = label;
                        else if (pos < p.C) gst(out + pos, (LT)label);
                    }
                }
            }
            running += rtot;
            if (direct) {
                flushed = running;
            } else {
                const uint32_t F = running & ~63u;  // complete 64-label units
                if (F > flushed) {
                    wave_sync_lds();
                    for (uint32_t q2 = flushed + lane; q2 < F; q2 += 64)
                        if (q2 < p.C) gst(out + q2, (LT)ring[q2 & smask]);
                    flushed = F;
                }
            }
            wave_sync_lds();  // the group's block slot and the ring are reused
        }
        if (lane == 0) ipos[T] = running;
        wave_sync_lds();
        for (uint32_t q2 = flushed + lane; q2 < running; q2 += 64)
            if (q2 < p.C) gst(out + q2, (LT)ring[q2 & smask]);
        if (c == 0 && g < nr) gst(p.counts + r0 + g, (uint32_t)(ipos[gfirst[g + 1]] - ipos[gfirst[g]]));
        if (lane == 0) gst(p.block_counts + rb, running);
        if (running > p.C) {  // rowblock overflow: its rows go to the direct pass
            unsigned long long k0 = 0;
            if (lane == 0) k0 = atomicAdd(&p.scalars[1], (unsigned long long)nr);
            k0 = (unsigned long long)__shfl((long long)k0, 0, 64);
            if (c == 0 && g < nr) gst(p.ovf_list + k0 + g, (uint32_t)(r0 + g));
        }
        wave_sync_lds();
    }
}

// ------------------------------------------------------------------------
// k_traverse_ptw: the traversal kernel for trees whose folded root's
// children are leaves or KIND_PACKT nodes -- any partitioner's shape (the
// greedy + relaxed trees of the reference's build scripts).  The rowblock
// phases of k_traverse_p2w, with one LANE per item in the rounds:
//   root phase -- group g reads the super-root's block at its row: up to 16
//                 children (WIDE: a second 64-byte half), their bits and
//                 positions (BRWT.cpp:30 + :43 for every child of the root);
//   items      -- the set (row, child) pairs in (row, child) order; a leaf
//                 child is an item of one label and no block;
//   rounds     -- lane L resolves item 64r + L: the 4 lanes of a group read
//                 the 64-byte KIND_PACKT blocks of the group's 4 items
//                 together (16 bytes each, one request per block), staged in
//                 LDS; the record's count byte places the item's labels (a
//                 wave scan), then the lane walks the DFS record over the PTW
//                 table in LDS and writes the labels -- in pre-order, the
//                 reference's order -- into the wave's ring;
//   flush      -- p2w's: 64-label units as full-line stores.
// MAXD: stack levels of the walk (>= the PACKT subtrees' height); WPB: waves
// per workgroup (the PTW table is staged once per workgroup).
// ------------------------------------------------------------------------
template <bool WIDE, uint32_t RING = 512>
struct PtwLayout {
    static constexpr uint32_t kItems = WIDE ? 256 : 128;  // 16 rows x R children
    static constexpr uint32_t kRing = RING;               // labels
    // items j | items k | row counts | group's first item | blocks (64 x 64 B) | ring
    static constexpr uint32_t kWords = kItems + kItems / 4 + 16 + 20 + 1024 + kRing;
};

// the labels of a KIND_PACKT record (masks from byte o on) into the ring
// (or, `direct`, the rowblock's temp region) from label position pos on
template <int MAXD, typename LT>
__device__ __forceinline__ void ptw_walk(const AS_LDS uint8_t *pb, uint32_t o, uint32_t node,
                                         const AS_LDS uint32_t *ntab, const AS_LDS uint16_t *etab,
                                         AS_LDS uint32_t *ring, uint32_t smask, uint32_t pos, bool direct,
                                         LT *out, uint32_t C, bool &overflow) {
    uint32_t nw = ntab[node];
    uint32_t m = pb[o++];
    if ((nw >> 24) > 8) m |= (uint32_t)pb[o++] << 8;
    uint32_t top = (nw & 0xFFFFu) | (m << 16);  // {first entry, children still to visit}
    uint32_t st[MAXD - 1];
#pragma unroll
    for (int k = 0; k < MAXD - 1; ++k) st[k] = 0;
    int sp = 0;
    while (true) {
        if ((top >> 16) == 0) {
            if (sp == 0) break;
            top = st[0];
#pragma unroll
            for (int k = 0; k < MAXD - 2; ++k) st[k] = st[k + 1];
            --sp;
            continue;
        }
        const uint32_t c = (uint32_t)__builtin_ctz(top >> 16);
        top &= ~(0x10000u << c);
        const uint32_t e = etab[(top & 0xFFFFu) + c];
        if (e & 0x8000u) {
            const uint32_t label = e & 0x7FFFu;
            if (!direct) ring[pos & smask] = label;
            else if (pos < C) gst(out + pos, (LT)label);
            ++pos;
            continue;
        }
        nw = ntab[e];
        uint32_t mw = pb[o++];
        if ((nw >> 24) > 8) mw |= (uint32_t)pb[o++] << 8;
        if (top >> 16) {  // the parent still has children to visit
            if (sp == MAXD - 1) {
                overflow = true;
                break;
            }
#pragma unroll
            for (int k = MAXD - 2; k > 0; --k) st[k] = st[k - 1];
            st[0] = top;
            ++sp;
        }
        top = (nw & 0xFFFFu) | (mw << 16);
    }
}

// The same walk for all 64 lanes of the wave at once, in lockstep and
// without per-lane branches (the branchy walk's exec-mask and loop handling
// measured more scalar than vector instructions per launch): each iteration
// takes one child of every lane's top frame; a leaf stores its column, an
// internal child pushes its frame (selects over the register stack) and an
// emptied frame is popped at the end of the iteration.  Lanes with no record
// (`live` false) idle.  Ring only (the `direct` rounds use ptw_walk).
template <int MAXD>
__device__ __forceinline__ void ptw_walk_wave(const AS_LDS uint8_t *pb, uint32_t o, uint32_t node, bool live,
                                              const AS_LDS uint32_t *ntab, const AS_LDS uint16_t *etab,
                                              AS_LDS uint32_t *ring, uint32_t smask, uint32_t pos, bool &overflow) {
    uint32_t nw = ntab[live ? node : 0u];
    uint32_t m = pb[o];
    const uint32_t w0 = (nw >> 24) > 8 ? 1u : 0u;
    m |= w0 ? (uint32_t)pb[o + 1] << 8 : 0u;
    o += 1 + w0;
    uint32_t top = live ? ((nw & 0xFFFFu) | (m << 16)) : 0u;
    uint32_t st[MAXD - 1];
#pragma unroll
    for (int k = 0; k < MAXD - 1; ++k) st[k] = 0;
    uint32_t sp = 0;
    bool done = !live || (top >> 16) == 0;
    while (__any(!done)) {
        const uint32_t mm = top >> 16;
        const uint32_t c = (uint32_t)__builtin_ctz(mm | 0x10000u);
        top &= ~(0x10000u << c);
        const uint32_t e = etab[done ? 0u : (top & 0xFFFFu) + c];
        const bool leaf = (e & 0x8000u) != 0;
        if (!done && leaf) ring[pos & smask] = e & 0x7FFFu;
        pos += (!done && leaf) ? 1u : 0u;
        const bool inner = !done && !leaf;
        const uint32_t nw2 = ntab[inner ? e : 0u];
        const uint32_t w2 = (nw2 >> 24) > 8 ? 1u : 0u;
        const uint32_t mw = (uint32_t)pb[o] | (w2 ? (uint32_t)pb[o + 1] << 8 : 0u);
        o += inner ? 1u + w2 : 0u;
        const bool push = inner && (top >> 16) != 0;
        overflow |= push && sp == (uint32_t)(MAXD - 1);
#pragma unroll
        for (int k = MAXD - 2; k > 0; --k) st[k] = push ? st[k - 1] : st[k];
        st[0] = push ? top : st[0];
        sp += push ? 1u : 0u;
        top = inner ? ((nw2 & 0xFFFFu) | (mw << 16)) : top;
        const bool pop = !done && (top >> 16) == 0 && sp > 0;  // (pushed frames are never empty)
        top = pop ? st[0] : top;
#pragma unroll
        for (int k = 0; k < MAXD - 2; ++k) st[k] = pop ? st[k + 1] : st[k];
        sp -= pop ? 1u : 0u;
        done = done || (top >> 16) == 0;
    }
}

template <bool NT, bool WIDE, int MAXD, int WPB, uint32_t RING = 512, typename LT = uint32_t>
__global__ __launch_bounds__(64 * WPB) void k_traverse_ptw(P2wParams p) {
    using Lay = PtwLayout<WIDE, RING>;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_ptw[];
    const uint32_t lane = threadIdx.x & 63, c = lane & 3, g = lane >> 2, gb = lane & ~3u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t i = threadIdx.x; i < p.table_words; i += blockDim.x) lds_ptw[i] = gld(p.table + i);
    __syncthreads();
    const AS_LDS uint32_t *tab = (const AS_LDS uint32_t *)lds_ptw;
    const uint32_t R = __builtin_amdgcn_readfirstlane(tab[0]), nI = __builtin_amdgcn_readfirstlane(tab[1]);
    const AS_LDS uint32_t *roots = tab + 4;
    const AS_LDS uint32_t *ntab = roots + 4 * R;
    const AS_LDS uint16_t *etab = (const AS_LDS uint16_t *)(ntab + nI);
    AS_LDS uint32_t *wbase = (AS_LDS uint32_t *)lds_ptw + ((p.table_words + 3) & ~3u) + wv * Lay::kWords;
    AS_LDS uint32_t *items_j = wbase;                                    // item position j
    AS_LDS uint8_t *items_k = (AS_LDS uint8_t *)(wbase + Lay::kItems);   // item child k
    AS_LDS uint32_t *rowcnt = wbase + Lay::kItems + Lay::kItems / 4;      // [16] labels per row
    AS_LDS uint32_t *gfirst = rowcnt + 16;                               // [17] group's first item; [16] = T
    AS_LDS uint32_t *slots = gfirst + 20;                                // lane L's 64-byte block: [16 L, 16 L + 16)
    AS_LDS uint32_t *ring = slots + 1024;                                // kRing labels
    AS_LDS uint32_t *mine = slots + 16 * lane;
    const AS_LDS uint8_t *pb = (const AS_LDS uint8_t *)mine;
    constexpr uint32_t smask = Lay::kRing - 1;
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    bool overflow = false;

    const uint64_t nblocks = (p.n + 15) / 16;
    const uint64_t wstride = (uint64_t)gridDim.x * WPB;
    for (uint64_t rb = (uint64_t)blockIdx.x * WPB + wv; rb < nblocks; rb += wstride) {
        const uint64_t r0 = rb * 16;
        const uint32_t nr = (uint32_t)(p.n - r0 < 16 ? p.n - r0 : 16);
        // LT: the temp region's label type (u16 when every label is < 2^16:
        // half the traversal's writes and the compaction's reads)
        LT *const out = reinterpret_cast<LT *>(p.temp) + rb * (uint64_t)p.C;

        // ---- root phase: the super-root's block at group g's row ----
        uint32_t row = kNone;
        if (r0 + g < p.n) {
            const uint64_t r = gld(p.rows + r0 + g);
            if (r < p.num_rows) row = (uint32_t)r;
            else if (c == 0) atomicOr(&p.scalars[2], 1ull);
        }
        uint4 qa = make_uint4(0, 0, 0, 0), qb = make_uint4(0, 0, 0, 0);
        const uint64_t rblk = p.root_base + (uint64_t)(row >> 5) * p.root_stride;
        if (row != kNone && 2 * c < R) qa = gld_at_nt<uint4, NT>(rblk + 16u * c);
        if (WIDE && row != kNone && 8 + 2 * c < R) qb = gld_at_nt<uint4, NT>(rblk + 64u + 16u * c);
        uint32_t P = 0, jj[4] = {0, 0, 0, 0};
        if (row != kNone) {
            const uint32_t t = row & 31, below = (1u << t) - 1u;
            const uint32_t k0 = 2 * c;
            const uint32_t b0 = k0 < R ? (qa.y >> t) & 1u : 0u, b1 = k0 + 1 < R ? (qa.w >> t) & 1u : 0u;
            jj[0] = qa.x + (uint32_t)__builtin_popcount(qa.y & below);
            jj[1] = qa.z + (uint32_t)__builtin_popcount(qa.w & below);
            P = (b0 | (b1 << 1)) << k0;
            if (WIDE) {
                const uint32_t b2 = 8 + k0 < R ? (qb.y >> t) & 1u : 0u, b3 = 9 + k0 < R ? (qb.w >> t) & 1u : 0u;
                jj[2] = qb.x + (uint32_t)__builtin_popcount(qb.y & below);
                jj[3] = qb.z + (uint32_t)__builtin_popcount(qb.w & below);
                P |= (b2 | (b3 << 1)) << (8 + k0);
            }
        }
        P = quad_or(P);
        // ---- items in (row, child) order ----
        {
            const uint32_t ng = (uint32_t)__builtin_popcount(P);
            uint32_t pre = 0;
#pragma unroll
            for (uint32_t b = 0; b < (WIDE ? 5u : 4u); ++b) {
                const uint64_t M = __ballot(c == 0 && ((ng >> b) & 1u));
                pre += (uint32_t)__popcll(M & ((1ull << gb) - 1ull)) << b;
            }
#pragma unroll
            for (uint32_t h = 0; h < (WIDE ? 4u : 2u); ++h) {
                const uint32_t k = (h < 2 ? 0u : 8u) + 2 * c + (h & 1u);
                if ((P >> k) & 1u) {
                    const uint32_t idx = pre + (uint32_t)__builtin_popcount(P & ((1u << k) - 1u));
                    items_j[idx] = jj[h];
                    items_k[idx] = (uint8_t)k;
                }
            }
            if (c == 0) {
                gfirst[g] = pre;
                rowcnt[g] = 0;
            }
            if (lane == 60) gfirst[16] = pre + ng;
        }
        wave_sync_lds();
        const uint32_t T = __builtin_amdgcn_readfirstlane(gfirst[16]);

        // ---- rounds: lane L resolves item ib + L ----
        uint32_t running = 0, flushed = 0;
        for (uint32_t ib = 0; ib < T; ib += 64) {
            // the group's 4 blocks, quarter c each (all 4 requests in flight together)
            uint4 q[4];
#pragma unroll
            for (uint32_t h = 0; h < 4; ++h) {
                q[h] = make_uint4(0, 0, 0, 0);
                const uint32_t ih = ib + 4 * g + h;
                if (ih < T) {
                    const uint32_t k = items_k[ih];
                    if (!(roots[4 * k + 3] >> 31)) {
                        const uint64_t ubase = (uint64_t)roots[4 * k] | ((uint64_t)roots[4 * k + 1] << 32);
                        q[h] = gld_at_nt<uint4, NT>(ubase + (uint64_t)(items_j[ih] / roots[4 * k + 2]) * kPack2Block +
                                                    16u * c);
                    }
                }
            }
#pragma unroll
            for (uint32_t h = 0; h < 4; ++h)
                ((AS_LDS u32x4_t *)(slots + 16 * (4 * g + h)))[c] = u32x4_t{q[h].x, q[h].y, q[h].z, q[h].w};
            wave_sync_lds();
            const uint32_t i = ib + lane;
            const bool act = i < T;
            uint32_t j = 0, k = 0;
            if (act) {
                j = items_j[i];
                k = items_k[i];
            }
            const uint32_t ent = roots[4 * k + 3];
            const bool blk = act && !(ent >> 31);
            uint32_t s = 0;
            if (blk) {
                const uint32_t t = j % roots[4 * k + 2];
                s = pb[t];
                if (pb[0] == 0) {
                    // spilled block: copy the position's record into the lane's
                    // slot (list = u16 start[S+1], then the records; <= 64 bytes)
                    const uint64_t la = ((uint64_t)mine[3] << 32) | mine[2];
                    const uint32_t s0 = gld_at<uint16_t>(la + 2ull * t), len = gld_at<uint16_t>(la + 2ull * t + 2) - s0;
                    AS_LDS uint8_t *pw = (AS_LDS uint8_t *)mine;
                    for (uint32_t o = 0; o < len; o += 4) {
                        uint8_t b4[4];
#pragma unroll
                        for (uint32_t e = 0; e < 4; ++e) b4[e] = o + e < len ? gld_at<uint8_t>(la + s0 + o + e) : 0;
#pragma unroll
                        for (uint32_t e = 0; e < 4; ++e)
                            if (o + e < len) pw[o + e] = b4[e];
                    }
                    s = 0;
                }
            }
            const uint32_t nl = blk ? (uint32_t)pb[s] : act ? 1u : 0u;  // the record's label count
            // the item's first label: a wave scan of the counts (lanes are in item order)
            uint32_t x = nl;
#pragma unroll
            for (uint32_t d = 1; d < 64; d <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
                if (lane >= d) x += y;
            }
            const uint32_t rtot = __builtin_amdgcn_readlane(x, 63);
            const uint32_t ibase = running + x - nl;
            if (act) {  // the item's row: the last group whose first item is <= i
                uint32_t gr = 0;
#pragma unroll
                for (uint32_t q2 = 1; q2 < 16; ++q2) gr = gfirst[q2] <= i ? q2 : gr;
                __hip_atomic_fetch_add((uint32_t *)(rowcnt + gr), nl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            }
            const bool direct = rtot + (running - flushed) > Lay::kRing;
            if (direct) {
                for (uint32_t q2 = flushed + lane; q2 < running; q2 += 64)
                    if (q2 < p.C) gst(out + q2, (LT)ring[q2 & smask]);
                wave_sync_lds();
            }
            if (!direct) {
                ptw_walk_wave<MAXD>(pb, s + 1, ent, blk, ntab, etab, ring, smask, ibase, overflow);
                if (act && !blk) ring[ibase & smask] = ent & 0x7FFFFFFFu;
            } else if (blk) {
                ptw_walk<MAXD, LT>(pb, s + 1, ent, ntab, etab, ring, smask, ibase, direct, out, p.C, overflow);
            } else if (act && ibase < p.C) {
                gst(out + ibase, (LT)(ent & 0x7FFFFFFFu));
            }
            running += rtot;
            if (direct) {
                flushed = running;
            } else {
                const uint32_t F = running & ~63u;  // complete 64-label units
                if (F > flushed) {
                    wave_sync_lds();
                    for (uint32_t q2 = flushed + lane; q2 < F; q2 += 64)
                        if (q2 < p.C) gst(out + q2, (LT)ring[q2 & smask]);
                    flushed = F;
                }
            }
            wave_sync_lds();  // the slots and the ring are reused
        }
        for (uint32_t q2 = flushed + lane; q2 < running; q2 += 64)
            if (q2 < p.C) gst(out + q2, (LT)ring[q2 & smask]);
        if (lane < nr) gst(p.counts + r0 + lane, rowcnt[lane]);
        if (lane == 0) gst(p.block_counts + rb, running);
        if (running > p.C) {  // rowblock overflow: its rows go to the direct pass
            unsigned long long k0 = 0;
            if (lane == 0) k0 = atomicAdd(&p.scalars[1], (unsigned long long)nr);
            k0 = (unsigned long long)__shfl((long long)k0, 0, 64);
            if (lane < nr) gst(p.ovf_list + k0 + lane, (uint32_t)(r0 + lane));
        }
        wave_sync_lds();
    }
    if (overflow) atomicOr(&p.scalars[2], 2ull);
}

// k_compact_blocks: output of k_traverse_p2w -> CSR.  16 lanes per 16-row
// block (4 blocks per wave): the rows' offsets (block offset + in-block
// prefix) and a contiguous copy of the block's labels, each lane's (up to 8)
// label reads issued before its stores.  Overflowing blocks (> C labels) are
// left to the direct pass.
template <bool BIG, typename LT = uint32_t>
__global__ __launch_bounds__(256) void k_compact_blocks(const uint32_t *__restrict__ counts,
                                                        const uint64_t *__restrict__ block_offsets,
                                                        const LT *__restrict__ temp, uint32_t C,
                                                        uint64_t *__restrict__ offsets, uint32_t *__restrict__ cols,
                                                        uint64_t n, const uint32_t *__restrict__ label_map,
                                                        uint32_t map_lds, uint64_t cap) {
    const LabelMap lmap = stage_label_map(label_map, map_lds);
    const uint32_t lane = threadIdx.x & 63, sub = lane & 15;
    const uint64_t nb = (n + 15) / 16;
    // launched before the host knows the total: a batch over the caller's
    // capacity writes nothing (the host then returns MBRWT_ERR_CAPACITY)
    if (gld(block_offsets + nb) > cap) return;
    const uint64_t stride = ((uint64_t)gridDim.x * blockDim.x) >> 4;
    for (uint64_t b = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4; b < nb; b += stride) {
        const uint64_t r0 = b * 16;
        const uint32_t nr = (uint32_t)(n - r0 < 16 ? n - r0 : 16);
        const uint64_t base = gld(block_offsets + b);
        const uint32_t mine = sub < nr ? gld(counts + r0 + sub) : 0u;
        // the first 128 labels are read before the block's total is known
        // (when the temp region holds C >= 128 words; always at the default
        // slot sizes): the label reads overlap the offset reads instead of
        // waiting behind them
        const LT *src = temp + b * (uint64_t)C;
        uint32_t v0[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) v0[k] = C >= 128 ? (uint32_t)gld(src + sub + 16 * k) : 0u;
        uint32_t x = mine;
#pragma unroll
        for (uint32_t d = 1; d < 16; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, d, 16);
            if (sub >= d) x += y;
        }
        const uint32_t total = (uint32_t)__shfl((int)x, 15, 16);
        if (sub < nr) gst(offsets + r0 + sub, base + (x - mine));
        if (sub == 0 && r0 + nr == n) gst(offsets + n, base + total);
        if (total > C) continue;
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {  // the first 128 labels
            const uint32_t i = sub + 16 * k;
            if (i < total) gst(cols + base + i, lmap(C < 128 ? (uint32_t)gld(src + i) : v0[k]));
        }
        // the rest, U labels per lane and round, every lane's reads issued
        // before its stores: U = 32 for large rows (BIG: e.g. 120 labels per
        // row at the RefSeq shape, 2.7 -> 2.1 ms per 10 M rows), 8 otherwise
        // (32 registers cost occupancy: 0.146 -> 0.201 ms at 8 labels per row)
        constexpr uint32_t U = BIG ? 32 : 8;
        for (uint32_t i0 = 128; i0 < total; i0 += 16 * U) {
            uint32_t v[U];
#pragma unroll
            for (uint32_t k = 0; k < U; ++k) {
                const uint32_t i = i0 + sub + 16 * k;
                v[k] = i < total ? (uint32_t)gld(src + i) : 0u;
            }
#pragma unroll
            for (uint32_t k = 0; k < U; ++k) {
                const uint32_t i = i0 + sub + 16 * k;
                if (i < total) gst(cols + base + i, lmap(v[k]));
            }
        }
    }
}

// CSR compaction of the label slots (rows with <= K labels).  A workgroup
// takes 256 consecutive rows; its threads walk the tile's contiguous output
// range [offsets[r0], offsets[r0+256]) so the stores are fully coalesced,
// find each position's row by a binary search over the tile's offsets in
// LDS, and read the slot labels (a row's labels are adjacent in its slot).
constexpr int kCompactTile = 256;

// k_compact_chunks: output of k_traverse_fast2 -> CSR.  The traversal packs
// the labels of the 8 rows of chunk ch back to back at temp + ch*8*K (rows
// with more than K labels left out for the overflow pass) and counts labels
// per row and per chunk; the scan runs over the chunk counts only.  Here 8
// lanes per chunk (8 chunks per wave) write the chunk's 8 row offsets (chunk
// offset + in-chunk prefix) and copy the packed labels; each lane issues its
// (up to 8) label reads before any store.  Contiguous reads and writes.
__global__ __launch_bounds__(256) void k_compact_chunks(const uint32_t *__restrict__ counts,
                                                        const uint64_t *__restrict__ chunk_offsets,
                                                        const uint32_t *__restrict__ temp, uint32_t K,
                                                        uint64_t *__restrict__ offsets, uint32_t *__restrict__ cols,
                                                        uint64_t n, const uint32_t *__restrict__ label_map,
                                                        uint32_t map_lds) {
    const LabelMap lmap = stage_label_map(label_map, map_lds);
    const uint32_t lane = threadIdx.x & 63, sub = lane & 7, gb = lane & ~7u;
    const uint64_t nch = (n + 7) / 8;
    const uint64_t stride = ((uint64_t)gridDim.x * blockDim.x) >> 3;
    for (uint64_t ch = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3; ch < nch; ch += stride) {
        const uint64_t r0 = ch * 8;
        const uint32_t nr = (uint32_t)(n - r0 < 8 ? n - r0 : 8);
        const uint64_t base = gld(chunk_offsets + ch);
        const uint32_t mine = sub < nr ? gld(counts + r0 + sub) : 0u;
        uint32_t cr[8];
#pragma unroll
        for (uint32_t r = 0; r < 8; ++r) cr[r] = (uint32_t)__shfl((int)mine, (int)(gb + r), 64);
        uint32_t pre[9], buf[9];
        pre[0] = buf[0] = 0;
#pragma unroll
        for (uint32_t r = 0; r < 8; ++r) {
            pre[r + 1] = pre[r] + cr[r];
            buf[r + 1] = buf[r] + (cr[r] <= K ? cr[r] : 0u);  // overflow rows hold no labels here
        }
        if (sub < nr) gst(offsets + r0 + sub, base + pre[sub]);
        if (sub == 0 && r0 + nr == n) gst(offsets + n, base + pre[nr]);
        const uint32_t stored = buf[nr];
        const uint32_t *src = temp + ch * 8 * K;
        if (stored == pre[nr]) {  // no overflow row in the chunk: packed label i is output label base + i
            for (uint32_t i0 = 0; i0 < stored; i0 += 64) {
                uint32_t v[8];
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k) {
                    const uint32_t i = i0 + sub + 8 * k;
                    v[k] = i < stored ? lmap(gld(src + i)) : 0u;
                }
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k) {
                    const uint32_t i = i0 + sub + 8 * k;
                    if (i < stored) gst(cols + base + i, v[k]);
                }
            }
            continue;
        }
        for (uint32_t i0 = 0; i0 < stored; i0 += 64) {
            uint32_t v[8];
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) {
                const uint32_t i = i0 + sub + 8 * k;
                v[k] = i < stored ? lmap(gld(src + i)) : 0u;
            }
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) {
                const uint32_t i = i0 + sub + 8 * k;
                if (i >= stored) continue;
                // the row owning packed label i (empty rows before it share its buf value)
                uint32_t prow = pre[0], brow = buf[0];
#pragma unroll
                for (uint32_t r = 1; r < 8; ++r)
                    if (r < nr && buf[r] <= i) {
                        prow = pre[r];
                        brow = buf[r];
                    }
                gst(cols + base + prow + (i - brow), v[k]);
            }
        }
    }
}

__global__ __launch_bounds__(kCompactTile) void k_compact(const uint64_t *__restrict__ offsets,
                                                          const uint32_t *__restrict__ temp, uint32_t K,
                                                          uint32_t *__restrict__ cols, uint64_t n,
                                                          const uint32_t *__restrict__ label_map, uint32_t map_lds) {
    __shared__ uint64_t soff[kCompactTile + 1];
    const LabelMap lmap = stage_label_map(label_map, map_lds);
    const uint32_t t = threadIdx.x;
    for (uint64_t tile = blockIdx.x; tile * kCompactTile < n; tile += gridDim.x) {
        const uint64_t r0 = tile * kCompactTile;
        const uint32_t rn = (uint32_t)((n - r0) < kCompactTile ? (n - r0) : kCompactTile);
        for (uint32_t i = t; i <= rn; i += kCompactTile) soff[i] = gld(offsets + r0 + i);
        __syncthreads();
        const uint64_t q0 = soff[0], q1 = soff[rn];
        for (uint64_t q = q0 + t; q < q1; q += kCompactTile) {
            uint32_t lo = 0, hi = rn;  // largest r with soff[r] <= q
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (soff[mid] <= q) lo = mid;
                else hi = mid;
            }
            const uint64_t c = soff[lo + 1] - soff[lo];
            if (c <= K) gst(cols + q, lmap(gld(temp + (r0 + lo) * K + (q - soff[lo]))));
        }
        __syncthreads();
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
            const DevNode ndv = gld(nodes + v);
            const DevNode *nd = &ndv;
            const uint32_t c = col_path[col * path_len + k];
            const uint64_t base = nd->base;
            if (nd->kind == KIND_PACKT) {  // the column's leaf below v (pre-order label), then one record walk
                uint32_t w = v;
                for (uint32_t kk = k; kk < path_len; ++kk) {
                    w = gld(nodes + w).first_child + col_path[col * path_len + kk];
                    if (gld(nodes + w).kind == KIND_LEAF) break;
                }
                const uint32_t want = gld(nodes + w).label;
                Pack2Block pb;
                pb.load(base, j, nd->stride);
                uint32_t hit = 0;
                (void)packt_walk(
                    nodes, v, [&](uint32_t o) { return pb.byte(o); }, pb.start(j % nd->stride),
                    [&](uint32_t label) { hit |= label == want; }, [](uint32_t) {});
                bit = (uint8_t)hit;
                break;
            }
            if (nd->kind == KIND_PACK2) {  // child c, its child c2, leaf c3: one record walk
                Pack2Block pb;
                pb.load(base, j, nd->stride);
                const uint32_t s = pb.start(j % nd->stride);
                const uint32_t m2 = pb.byte(s);
                if ((m2 >> c) & 1u) {
                    const uint32_t c2 = col_path[col * path_len + k + 1], c3 = col_path[col * path_len + k + 2];
                    const uint32_t i = (uint32_t)__builtin_popcount(m2 & ((1u << c) - 1u));
                    const uint32_t m1 = pb.byte(s + 1 + i);
                    if ((m1 >> c2) & 1u) {
                        uint32_t o = s + 1 + (uint32_t)__builtin_popcount(m2);  // leaf masks of earlier children
                        for (uint32_t q = 0; q < i; ++q) o += (uint32_t)__builtin_popcount(pb.byte(s + 1 + q));
                        o += (uint32_t)__builtin_popcount(m1 & ((1u << c2) - 1u));
                        bit = (uint8_t)((pb.byte(o) >> c3) & 1u);
                    }
                }
                break;
            }
            if (nd->kind == KIND_PACK) {  // child c is a MASK8 node: its bit, then its mask
                PackBlock pb;
                pb.load(base, j);
                const uint32_t t = j % kPackSpan;
                uint32_t o = 0;
                for (uint32_t q = 0; q < c; ++q) o += (uint32_t)__builtin_popcount(pb.bits(q));
                const uint32_t bc = pb.bits(c);
                if ((bc >> t) & 1u) {
                    const uint32_t m = pb.mask(o + (uint32_t)__builtin_popcount(bc & ((1u << t) - 1u)));
                    bit = (uint8_t)((m >> col_path[col * path_len + k + 1]) & 1u);
                }
                break;
            }
            if (nd->kind == KIND_PLANE) {
                const uint2 rb = gld_at<uint2>(base + (uint64_t)(j >> 5) * nd->stride + 8u * c);
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
                if (nd->kind == KIND_MASK8) m = gld_at<uint8_t>(base + j);
                else if (nd->kind == KIND_MASK16) m = gld_at<uint16_t>(base + 2ull * j);
                else if (nd->kind == KIND_MASK32) m = gld_at<uint32_t>(base + 4ull * j);
                else m = gld_at<uint64_t>(base + 8ull * j);
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
using GroupFn = void (*)(TravParams, uint32_t);

// A traversal launch: the lane-per-row kernel or the group kernel.
struct Trav {
    const void *fn = nullptr;
    TravFn lane_fn = nullptr;
    GroupFn group_fn = nullptr;
    uint32_t G = 1;  // lanes per row
    bool fast = false;
    const char *name = "k_traverse_group";
    explicit operator bool() const { return fn != nullptr; }
};

uint32_t auto_slots(const Ctx &c);

template <int MODE>
Trav pick_traverse(const Ctx &c) {
    const uint32_t depth = c.tree.stack_depth, max_arity = c.tree.max_arity;
    Trav t;
    const int kv = c.kernel_variant;
    const bool p2 = c.tree.has_pack2;
    if (MODE == MODE_SLOTS && c.tree.fast_shape && c.tree.lds_complete && (kv == 0 || (kv >= 17 && kv <= 23)) &&
        (!p2 || (c.tree.push_frames <= 1 && !c.tree.has_mask_children))) {
        // k_traverse_fast2; 17/18 force plain / non-temporal block reads, the
        // default uses non-temporal reads on images larger than 1 GiB (+2.6 %)
        const bool nt = kv == 18 || kv == 20 || (kv == 0 && c.tree.image_bytes > (1ull << 30));
        const bool smallk = auto_slots(c) == kStageLabels;
        t.G = 4;
        t.fast = true;
        t.name = p2 ? "k_traverse_fast2/pack2" : "k_traverse_fast2";
#define FAST2(P)                                                                                          \
    if (smallk) t.lane_fn = nt ? (TravFn)k_traverse_fast2<true, true, P> : (TravFn)k_traverse_fast2<false, true, P>; \
    else t.lane_fn = nt ? (TravFn)k_traverse_fast2<true, false, P> : (TravFn)k_traverse_fast2<false, false, P>;
        if (p2) {
            FAST2(true)
        } else {
            FAST2(false)
        }
#undef FAST2
        t.fn = reinterpret_cast<const void *>(t.lane_fn);
        return t;
    }
    if (c.kernel_variant == 1 || c.tree.has_packt) {  // lane-per-row kernel (A/B; the general kernel of KIND_PACKT trees)
        const bool wide = max_arity > 32;
        t.name = "k_traverse";
#define PICK(D)                                                                                      \
    if (depth <= D) {                                                                                \
        t.lane_fn = wide ? (TravFn)k_traverse<D, uint64_t, MODE> : (TravFn)k_traverse<D, uint32_t, MODE>; \
        t.fn = reinterpret_cast<const void *>(t.lane_fn);                                            \
        return t;                                                                                    \
    }
        PICK(4)
        PICK(8)
        PICK(16)
        PICK(32)
#undef PICK
        return t;
    }
    // group kernel: CPL children per lane, G = pow2ceil(ceil(max_arity / CPL)) lanes per row;
    // variants 5/6 request a higher occupancy (waves per SIMD) from the register allocator
    // default (and the fast variants on trees they do not fit): 2 children per lane, 8 waves/SIMD
    const int v = (c.kernel_variant == 0 || c.kernel_variant >= 11) ? 5 : c.kernel_variant;  // 17/18: fast2 only
    const int cpl = v == 2 ? 1 : (v == 4 || v == 6) ? 4 : 2;
    const int wpe = (v == 5 || v == 10) ? 8 : v == 6 ? 6 : 1;  // (v == 10 past depth 8 runs as 5)
    const uint32_t need = (max_arity + cpl - 1) / cpl;
    uint32_t G = 1;
    while (G < need) G <<= 1;
    t.G = G;
#define PICKG(D, CPLV, W)                                                                          \
    if (depth <= D && cpl == CPLV && wpe == W) {                                                   \
        t.group_fn = max_arity <= 32 ? (GroupFn)k_traverse_group<D, CPLV, uint32_t, MODE, W>       \
                                     : (GroupFn)k_traverse_group<D, CPLV, uint64_t, MODE, W>;      \
        t.fn = reinterpret_cast<const void *>(t.group_fn);                                         \
        return t;                                                                                  \
    }
#define PICKD(CPLV, W) PICKG(4, CPLV, W) PICKG(8, CPLV, W) PICKG(16, CPLV, W) PICKG(32, CPLV, W)
    PICKD(2, 8)
#undef PICKD
#undef PICKG
    return t;
}

// node records staged in LDS: the first min(kLdsNodes, last non-leaf + 1)
uint32_t lds_node_count(const Ctx &c) {
    return (uint32_t)std::min<size_t>({c.tree.nodes.size(), (size_t)kLdsNodes, (size_t)c.tree.lds_records});
}

size_t lds_bytes(const Ctx &c, const Trav &t) {
    if (!t.group_fn && !t.fast) return 0;
    // label stages (+ one 64-byte PACK block per group for fast2) + node records
    return (size_t)(256 / t.G) * kStageLabels * sizeof(uint32_t) + (t.fast ? 64 * kPackBlock : 0) +
           (size_t)lds_node_count(c) * sizeof(CNode);
}

int grid_for(const Ctx &c, const Trav &t, uint64_t n) {
    int dev_cus = 0;
    (void)hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, c.device);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, t.fn, 256, lds_bytes(c, t)) != hipSuccess || per_cu <= 0)
        per_cu = 4;
    const uint64_t resident = (uint64_t)std::max(1, dev_cus) * (uint64_t)per_cu;
    // fast: 64 groups x 8-row chunks (x 2 contexts for fast3)
    const uint64_t rows_per_block = t.fast ? 512 : 256 / t.G;
    const uint64_t need = (n + rows_per_block - 1) / rows_per_block;
    return (int)std::max<uint64_t>(1, std::min(need, resident));
}

hipError_t launch(const Ctx &c, const Trav &t, uint64_t n, hipStream_t s, const TravParams &p) {
    const int grid = grid_for(c, t, n);
    if (t.group_fn) hipLaunchKernelGGL(t.group_fn, dim3(grid), dim3(256), lds_bytes(c, t), s, p, t.G);
    else hipLaunchKernelGGL(t.lane_fn, dim3(grid), dim3(256), lds_bytes(c, t), s, p);
    return hipGetLastError();
}

// label-map entries the compaction kernels stage in LDS (0: identity or too large)
uint32_t label_map_lds(const Ctx &c) {
    const size_t m = c.tree.label_perm.size();
    return (c.d_label_map && m <= kMapLdsMax) ? (uint32_t)m : 0u;
}

uint32_t auto_slots(const Ctx &c) {
    if (c.slot_labels) return c.slot_labels;
    const double mean = c.tree.num_rows ? (double)c.tree.num_relations / (double)c.tree.num_rows : 0.0;
    uint32_t k = kStageLabels;  // >= the LDS stage of the group kernel
    while (k < 2.0 * mean + 8.0 && k < 1024) k <<= 1;
    return k;
}

TravParams base_params(const Ctx &c) {
    TravParams p{};
    p.nodes = c.d_nodes;
    p.cnodes = c.d_cnodes;
    p.n_lds = lds_node_count(c);
    p.folded = c.tree.folded ? 1u : 0u;
    p.num_rows = c.tree.num_rows;
    p.scalars = reinterpret_cast<unsigned long long *>(c.d_scalars);
    p.label_map = c.d_label_map;
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

// k_traverse_p2w for this context?  Default for trees with a P2W table;
// MBRWT_OPT_KERNEL 19 / 20 force plain / non-temporal reads (A/B; 17 / 18
// force k_traverse_fast2).
using P2wFn = void (*)(P2wParams);
static P2wFn p2w_kernel(const Ctx &c) {
    const int kv = c.kernel_variant;
    if (c.tree.p2w_table.empty() || !c.d_p2w || !(kv == 0 || kv == 19 || kv == 20)) return nullptr;
    const bool big = c.tree.image_bytes > (1ull << 30);
    switch (kv) {
    default:  // u16 temp labels when they fit (p2w_label16)
        if (c.tree.num_columns <= 0x10000u) return big ? k_traverse_p2w<true, uint16_t> : k_traverse_p2w<false, uint16_t>;
        return big ? k_traverse_p2w<true> : k_traverse_p2w<false>;
    }
}

// the default p2w kernel stores u16 temp labels (label indices < num_columns)
static bool p2w_label16(const Ctx &c) { return c.kernel_variant == 0 && c.tree.num_columns <= 0x10000u; }

static uint32_t p2w_ring(const Ctx &c) {
    (void)c;
    return 512;
}

static size_t p2w_lds_bytes(const Ctx &c) {
    return ((c.tree.p2w_table.size() + 3) & ~size_t(3)) * 4 + 4 * (size_t)(kP2wWaveWords + p2w_ring(c)) * 4;
}

// k_traverse_ptw for this context?  Default for trees with a PTW table
// (MBRWT_OPT_KERNEL 0 or 24..30): 24 plain reads, 25 non-temporal, 26/27 the
// same with 8 waves per workgroup, 28/29 with 16 (512-label rings: LDS holds
// 16 waves per CU); 30 and the default: 7 waves per workgroup with a
// 256-label ring (21 waves per CU; 2.27 vs 2.47 ms at the greedy + relax shape).
struct PtwPick {
    P2wFn fn = nullptr;
    uint32_t wpb = 4;
    uint32_t ring = 512;
    bool wide = false;
    bool label16 = false;  // u16 temp labels (the default 7-wave kernel; PTW columns are < 2^15)
};
template <bool NT, bool WIDE, int MAXD>
static P2wFn ptw_fn(uint32_t wpb) {
    (void)wpb;  // (the default 7-wave kernel only; the r02 wave-count variants were retired)
    return k_traverse_ptw<NT, WIDE, MAXD, 7, 256, uint16_t>;
}
static PtwPick ptw_kernel(const Ctx &c) {
    PtwPick r;
    const int kv = c.kernel_variant;
    const auto &t = c.tree.ptw_table;
    if (t.empty() || !c.d_ptw || !(kv == 0 || (kv >= 24 && kv <= 30))) return r;
    const bool nt = kv == 0 || kv == 30 ? c.tree.image_bytes > (1ull << 30) : (kv & 1) != 0;
    r.wpb = (kv == 0 || kv == 30) ? 7 : kv >= 28 ? 16 : kv >= 26 ? 8 : 4;  // default: 7 waves, 256-label ring
    r.ring = r.wpb == 7 ? 256 : 512;
    r.label16 = r.wpb == 7;
    r.wide = t[0] > 8;
    const bool deep = t[3] > 4;
#define PTW(NTV, W, D) if (nt == NTV && r.wide == W && deep == D) r.fn = ptw_fn<NTV, W, D ? 8 : 4>(r.wpb);
    PTW(false, false, false) PTW(false, false, true) PTW(false, true, false) PTW(false, true, true)
    PTW(true, false, false) PTW(true, false, true) PTW(true, true, false) PTW(true, true, true)
#undef PTW
    return r;
}

const char *traverse_kernel_name(const Ctx &c) {
    if (c.rows.ready && c.kernel_variant == 0) return c.rows.var ? "k_var_decode" : "k_traverse_rows";
    if (c.nodes_freed) return "";
    if (ptw_kernel(c).fn) return "k_traverse_ptw";
    if (p2w_kernel(c)) return "k_traverse_p2w";
    const Trav t = pick_traverse<MODE_SLOTS>(c);
    return t ? t.name : "";
}

// get_rows through k_traverse_p2w: rowblocks of 16 rows, each written to its
// own temp region of C = 16 K labels; one scan over the rowblock totals; the
// compaction; the direct pass for overflowing rowblocks.
// (k_traverse_ptw: the same driver over the PTW table, `wpb` waves per workgroup)
struct RowblockKernel {
    P2wFn fn;
    const uint32_t *table;
    uint32_t table_words;
    size_t lds;
    uint32_t wpb;
    bool final_columns;  // the kernel emits global columns (k_traverse_ptw): no label map afterwards
    bool label16;        // u16 temp labels
};
static int run_get_rows_p2w(Ctx &c, const RowblockKernel &kr, const uint64_t *d_rows, uint64_t n,
                            uint64_t *d_offsets, uint32_t *d_cols, uint64_t cap, uint64_t *needed, hipStream_t s) {
    const P2wFn kfn = kr.fn;
    const uint32_t K = auto_slots(c);
    const uint32_t C = 16 * K;
    const Trav fn_direct = pick_traverse<MODE_DIRECT>(c);
    if (!fn_direct) {
        set_error("tree deeper than 32 levels of internal nodes");
        return MBRWT_ERR_UNSUPPORTED;
    }
    int rc;
    const uint64_t nb = (n + 15) / 16;
    // counts: n row counts | nb+1 block counts | (8-byte aligned) nb+1 block offsets
    const uint64_t bc_off = n, bo_off = ((bc_off + nb + 1) * sizeof(uint32_t) + 7) / 8 * 8;
    if ((rc = ensure(c.ws_temp, nb * (uint64_t)C * (kr.label16 ? 2u : 4u)))) return rc;
    if ((rc = ensure(c.ws_counts, bo_off + (nb + 1) * sizeof(uint64_t)))) return rc;
    if ((rc = ensure(c.ws_ovf, n * sizeof(uint32_t)))) return rc;
    uint32_t *d_counts = reinterpret_cast<uint32_t *>(c.ws_counts.buf);
    uint32_t *d_block_counts = d_counts + bc_off;
    uint64_t *d_block_offsets = reinterpret_cast<uint64_t *>(reinterpret_cast<uint8_t *>(c.ws_counts.buf) + bo_off);
    hipcub::TransformInputIterator<uint64_t, U32ToU64, const uint32_t *> it(d_block_counts, U32ToU64());
    size_t scan_bytes = 0;
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, it, d_block_offsets, nb + 1, s));
    if ((rc = ensure(c.ws_scan, scan_bytes))) return rc;

    const DevNode &root = c.tree.nodes[0];
    P2wParams p{};
    p.rows = d_rows;
    p.n = n;
    p.num_rows = c.tree.num_rows;
    p.root_base = root.base;
    p.root_stride = root.stride;
    p.table_words = kr.table_words;
    p.table = kr.table;
    p.C = C;
    p.S = p2w_ring(c);
    p.temp = reinterpret_cast<uint32_t *>(c.ws_temp.buf);
    p.counts = d_counts;
    p.block_counts = d_block_counts;
    p.ovf_list = reinterpret_cast<uint32_t *>(c.ws_ovf.buf);
    p.scalars = reinterpret_cast<unsigned long long *>(c.d_scalars);

    const size_t lds = kr.lds;
    const uint32_t threads = 64 * kr.wpb;
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
        c.rb_fn = reinterpret_cast<const void *>(kfn);
        c.rb_lds = lds;
        c.rb_threads = threads;
        c.rb_blocks = std::max(1, dev_cus) * per_cu;
    }
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((nb + kr.wpb - 1) / kr.wpb, (uint64_t)c.rb_blocks));

    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 8 * sizeof(uint64_t), s));
    MBRWT_HIP(hipMemsetAsync(d_block_counts + nb, 0, sizeof(uint32_t), s));
    if (c.timing) MBRWT_HIP(hipEventRecord(c.ev0, s));
    hipLaunchKernelGGL(kfn, dim3((unsigned)grid), dim3(threads), lds, s, p);
    MBRWT_HIP(hipGetLastError());
    if (c.timing) MBRWT_HIP(hipEventRecord(c.ev1, s));
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(c.ws_scan.buf, scan_bytes, it, d_block_offsets, nb + 1, s));
    // the compaction is queued right behind the scan, before the host learns
    // the total (one synchronisation per call, after it; the kernel checks
    // the capacity itself)
    const uint32_t map_lds = kr.final_columns ? 0u : label_map_lds(c);
    // one 16-lane group per rowblock and no grid-stride rounds: with 8192
    // workgroups each wave walked ~15 rowblocks through two dependent memory
    // latencies each
    const uint64_t g = std::min<uint64_t>((nb + 15) / 16, 1u << 20);
    const bool big = c.tree.num_rows && (double)c.tree.num_relations > 32.0 * (double)c.tree.num_rows;
    const uint32_t *lm = kr.final_columns ? nullptr : (const uint32_t *)c.d_label_map;
    if (kr.label16) {
        auto *cfn = big ? k_compact_blocks<true, uint16_t> : k_compact_blocks<false, uint16_t>;
        hipLaunchKernelGGL(cfn, dim3((unsigned)g), dim3(256), map_lds * 4, s, d_counts, d_block_offsets,
                           reinterpret_cast<const uint16_t *>(p.temp), C, d_offsets, d_cols, n, lm, map_lds, cap);
    } else
        hipLaunchKernelGGL(big ? k_compact_blocks<true> : k_compact_blocks<false>, dim3((unsigned)g), dim3(256),
                           map_lds * 4, s, d_counts, d_block_offsets, (const uint32_t *)p.temp, C, d_offsets, d_cols, n,
                           lm, map_lds, cap);
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipMemcpyAsync(c.d_scalars, d_block_offsets + nb, sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
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
    if (ovf) {
        TravParams q = base_params(c);
        q.rows = d_rows;
        q.n = ovf;
        q.K = K;
        q.slot_list = p.ovf_list;
        q.offsets = d_offsets;
        q.cols = d_cols;
        MBRWT_HIP(launch(c, fn_direct, ovf, s, q));
    }
    return MBRWT_OK;
}

int run_get_rows(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets, uint32_t *d_cols, uint64_t cap,
                 uint64_t *needed, hipStream_t s) {
    if (c.rows.ready && c.kernel_variant == 0) return rows_get_rows(c, d_rows, n, d_offsets, d_cols, cap, needed, s);
    if (c.nodes_freed) {
        set_error("kernel variant needs the node image (layout rows)");
        return MBRWT_ERR_UNSUPPORTED;
    }
    c.rows_sc_dirty = true;  // the node kernels reuse ws_counts
    if (!c.shards.empty()) return sharded_get_rows(c, d_rows, n, d_offsets, d_cols, cap, needed, s);
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
    if (n > 0x7FFFFFF0ull) {  // u32 slot arithmetic in the kernels
        set_error("batch larger than 2^31 rows");
        return MBRWT_ERR_UNSUPPORTED;
    }
    if (const PtwPick pk = ptw_kernel(c); pk.fn) {
        const size_t words = c.tree.ptw_table.size();
        const size_t per_wave = pk.ring == 256 ? (pk.wide ? PtwLayout<true, 256>::kWords : PtwLayout<false, 256>::kWords)
                                               : (pk.wide ? PtwLayout<true>::kWords : PtwLayout<false>::kWords);
        const RowblockKernel kr{pk.fn, c.d_ptw, (uint32_t)words, ((words + 3) & ~size_t(3)) * 4 + pk.wpb * per_wave * 4,
                                pk.wpb, true, pk.label16};
        return run_get_rows_p2w(c, kr, d_rows, n, d_offsets, d_cols, cap, needed, s);
    }
    if (const P2wFn kfn = p2w_kernel(c)) {
        const RowblockKernel kr{kfn, c.d_p2w, (uint32_t)c.tree.p2w_table.size(), p2w_lds_bytes(c), 4, false,
                                p2w_label16(c)};
        return run_get_rows_p2w(c, kr, d_rows, n, d_offsets, d_cols, cap, needed, s);
    }
    const uint32_t K = auto_slots(c);
    const Trav fn = pick_traverse<MODE_SLOTS>(c);
    const Trav fn_direct = pick_traverse<MODE_DIRECT>(c);
    if (!fn || !fn_direct) {
        set_error("tree deeper than 32 levels of internal nodes");
        return MBRWT_ERR_UNSUPPORTED;
    }
    int rc;
    const uint64_t nch = (n + 7) / 8;
    // counts: n+1 row counts | nch+1 chunk counts | (8-byte aligned) nch+1 chunk offsets
    const uint64_t cc_off = n + 1, co_off = ((cc_off + nch + 1) * sizeof(uint32_t) + 7) / 8 * 8;
    if ((rc = ensure(c.ws_temp, n * K * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(c.ws_counts, co_off + (nch + 1) * sizeof(uint64_t)))) return rc;
    if ((rc = ensure(c.ws_ovf, n * sizeof(uint32_t)))) return rc;
    uint32_t *d_counts = reinterpret_cast<uint32_t *>(c.ws_counts.buf);
    uint32_t *d_chunk_counts = d_counts + cc_off;
    uint64_t *d_chunk_offsets = reinterpret_cast<uint64_t *>(reinterpret_cast<uint8_t *>(c.ws_counts.buf) + co_off);
    // scan input: the row counts (general kernels) or the chunk counts (fast2)
    hipcub::TransformInputIterator<uint64_t, U32ToU64, const uint32_t *> it(fn.fast ? d_chunk_counts : d_counts,
                                                                            U32ToU64());
    uint64_t *scan_out = fn.fast ? d_chunk_offsets : d_offsets;
    const uint64_t scan_n = (fn.fast ? nch : n) + 1;
    size_t scan_bytes = 0;
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, it, scan_out, scan_n, s));
    if ((rc = ensure(c.ws_scan, scan_bytes))) return rc;

    TravParams p = base_params(c);
    p.rows = d_rows;
    p.n = n;
    p.K = K;
    p.temp = reinterpret_cast<uint32_t *>(c.ws_temp.buf);
    p.counts = d_counts;
    p.chunk_counts = d_chunk_counts;
    p.ovf_list = reinterpret_cast<uint32_t *>(c.ws_ovf.buf);

    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 8 * sizeof(uint64_t), s));
    MBRWT_HIP(hipMemsetAsync(fn.fast ? d_chunk_counts + nch : d_counts + n, 0, sizeof(uint32_t), s));
    if (c.timing) MBRWT_HIP(hipEventRecord(c.ev0, s));
    MBRWT_HIP(launch(c, fn, n, s, p));
    if (c.timing) MBRWT_HIP(hipEventRecord(c.ev1, s));
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(c.ws_scan.buf, scan_bytes, it, scan_out, scan_n, s));
    MBRWT_HIP(hipMemcpyAsync(c.d_scalars, scan_out + scan_n - 1, sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
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
        const uint32_t map_lds = label_map_lds(c);
        if (fn.fast) {  // chunk-packed output (k_traverse_fast2)
            const uint64_t g = std::min<uint64_t>(((n + 7) / 8 + 31) / 32, 1u << 20);  // no grid-stride rounds
            hipLaunchKernelGGL(k_compact_chunks, dim3((unsigned)g), dim3(256), map_lds * 4, s, d_counts, d_chunk_offsets, p.temp,
                               K, d_offsets, d_cols, n, (const uint32_t *)c.d_label_map, map_lds);
        } else {
            const uint64_t g = std::min<uint64_t>((n + kCompactTile - 1) / kCompactTile, 16384);
            hipLaunchKernelGGL(k_compact, dim3((unsigned)g), dim3(kCompactTile), map_lds * 4, s, d_offsets, p.temp, K,
                               d_cols, n, (const uint32_t *)c.d_label_map, map_lds);
        }
        MBRWT_HIP(hipGetLastError());
    }
    if (ovf) {
        TravParams q = p;
        q.n = ovf;
        q.slot_list = p.ovf_list;
        q.offsets = d_offsets;
        q.cols = d_cols;
        MBRWT_HIP(launch(c, fn_direct, ovf, s, q));
    }
    return MBRWT_OK;
}

int run_count_work(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *visits, uint64_t *labels, hipStream_t s) {
    if (c.nodes_freed) return rows_count_work(c, d_rows, n, visits, labels, s);
    if (!c.shards.empty()) return sharded_count_work(c, d_rows, n, visits, labels, s);
    if (c.tree.nodes.empty()) return n ? MBRWT_ERR_RANGE : MBRWT_OK;
    const Trav fn = pick_traverse<MODE_WORK>(c);
    if (!fn) return MBRWT_ERR_UNSUPPORTED;
    TravParams p = base_params(c);
    p.rows = d_rows;
    p.n = n;
    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 8 * sizeof(uint64_t), s));
    if (n) MBRWT_HIP(launch(c, fn, n, s, p));
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (c.h_scalars[2] & 1) return MBRWT_ERR_RANGE;
    if (c.h_scalars[2] & 2) return MBRWT_ERR_UNSUPPORTED;
    if (visits) *visits = c.h_scalars[3];
    if (labels) *labels = c.h_scalars[4];
    return MBRWT_OK;
}

int run_count_labels(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_counts, hipStream_t s) {
    if (c.rows.ready) return rows_count_labels(c, d_rows, n, d_counts, s);
    if (!c.shards.empty()) return sharded_count_labels(c, d_rows, n, d_counts, s);
    if (c.tree.num_columns) MBRWT_HIP(hipMemsetAsync(d_counts, 0, c.tree.num_columns * sizeof(uint64_t), s));
    if (c.tree.nodes.empty()) return n ? MBRWT_ERR_RANGE : MBRWT_OK;
    const Trav fn = pick_traverse<MODE_COUNT>(c);
    if (!fn) return MBRWT_ERR_UNSUPPORTED;
    TravParams p = base_params(c);
    p.rows = d_rows;
    p.n = n;
    p.label_counts = reinterpret_cast<unsigned long long *>(d_counts);
    MBRWT_HIP(hipMemsetAsync(c.d_scalars, 0, 8 * sizeof(uint64_t), s));
    if (n) MBRWT_HIP(launch(c, fn, n, s, p));
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, c.d_scalars, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (c.h_scalars[2] & 1) return MBRWT_ERR_RANGE;
    if (c.h_scalars[2] & 2) return MBRWT_ERR_UNSUPPORTED;
    return MBRWT_OK;
}

int run_get_batch(Ctx &c, const uint64_t *d_rows, const uint64_t *d_cols, uint64_t n, uint8_t *d_out, hipStream_t s) {
    if (c.nodes_freed) return rows_get_batch(c, d_rows, d_cols, n, d_out, s);
    if (!c.shards.empty()) return sharded_get_batch(c, d_rows, d_cols, n, d_out, s);
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

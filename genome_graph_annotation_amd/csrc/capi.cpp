// capi.cpp -- the extern "C" boundary of libmbrwt (include/mbrwt.h).
// Never throws across the ABI; every failure is an MBRWT_* status plus a
// thread-local message (mbrwt_last_error_message).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>

#include "mbrwt_internal.hpp"

namespace mbrwt {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int hip_fail(hipError_t e, const char *what) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    (void)hipGetLastError();  // clear the sticky non-fatal error
    return (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? MBRWT_ERR_NOMEM : MBRWT_ERR_DEVICE;
}

static int init_query_state(Ctx &c);

static int upload_tables(Ctx &c) {
    Tree &t = c.tree;
    if (!t.nodes.empty()) {
        MBRWT_HIP(hipMalloc(&c.d_nodes, t.nodes.size() * sizeof(DevNode)));
        MBRWT_HIP(hipMemcpy(c.d_nodes, t.nodes.data(), t.nodes.size() * sizeof(DevNode), hipMemcpyHostToDevice));
        std::vector<CNode> cn(t.nodes.size());
        for (size_t i = 0; i < cn.size(); ++i) {
            if (t.nodes[i].base >> 48) {
                set_error("device address above 2^48");
                return MBRWT_ERR_UNSUPPORTED;
            }
            cn[i] = compact(t.nodes[i]);
        }
        MBRWT_HIP(hipMalloc(&c.d_cnodes, cn.size() * sizeof(CNode)));
        MBRWT_HIP(hipMemcpy(c.d_cnodes, cn.data(), cn.size() * sizeof(CNode), hipMemcpyHostToDevice));
    }
    if (!t.label_perm.empty()) {
        MBRWT_HIP(hipMalloc(&c.d_label_map, t.label_perm.size() * 4));
        MBRWT_HIP(hipMemcpy(c.d_label_map, t.label_perm.data(), t.label_perm.size() * 4, hipMemcpyHostToDevice));
    }
    if (!t.p2w_table.empty()) {
        MBRWT_HIP(hipMalloc(&c.d_p2w, t.p2w_table.size() * 4));
        MBRWT_HIP(hipMemcpy(c.d_p2w, t.p2w_table.data(), t.p2w_table.size() * 4, hipMemcpyHostToDevice));
    }
    if (!t.ptw_table.empty()) {
        MBRWT_HIP(hipMalloc(&c.d_ptw, t.ptw_table.size() * 4));
        MBRWT_HIP(hipMemcpy(c.d_ptw, t.ptw_table.data(), t.ptw_table.size() * 4, hipMemcpyHostToDevice));
    }
    if (!t.col_path.empty()) {
        MBRWT_HIP(hipMalloc(&c.d_col_path, t.col_path.size()));
        MBRWT_HIP(hipMemcpy(c.d_col_path, t.col_path.data(), t.col_path.size(), hipMemcpyHostToDevice));
    }
    if (!t.col_leaf.empty()) {
        MBRWT_HIP(hipMalloc(&c.d_col_leaf, t.col_leaf.size() * 4));
        MBRWT_HIP(hipMemcpy(c.d_col_leaf, t.col_leaf.data(), t.col_leaf.size() * 4, hipMemcpyHostToDevice));
    }
    return init_query_state(c);
}

// the per-context query state: status scalars, timing events, workspace fence
static int init_query_state(Ctx &c) {
    MBRWT_HIP(hipHostMalloc(reinterpret_cast<void **>(&c.h_scalars), 8 * sizeof(uint64_t), hipHostMallocDefault));
    MBRWT_HIP(hipMalloc(&c.d_scalars, 8 * sizeof(uint64_t)));
    MBRWT_HIP(hipEventCreate(&c.ev0));
    MBRWT_HIP(hipEventCreate(&c.ev1));
    MBRWT_HIP(create_fence(c.fence));
    return MBRWT_OK;
}

static std::mutex g_clone_mu;  // Ctx::clones / Ctx::released of every image owner

static void release(Ctx *c) {
    if (!c) return;
    if (!c->image_owner) {
        std::lock_guard<std::mutex> lk(g_clone_mu);
        if (c->clones > 0) {  // freed with its last clone
            c->released = true;
            return;
        }
    }
    for (Ctx *sc : c->shards) release(sc);
    (void)hipSetDevice(c->device);
    if (!c->image_owner) {  // the image: only its owner frees it
        free_tree(c->tree);
        free_rows(c->rows);
        if (c->d_nodes) (void)hipFree(c->d_nodes);
        if (c->d_cnodes) (void)hipFree(c->d_cnodes);
        if (c->d_p2w) (void)hipFree(c->d_p2w);
        if (c->d_ptw) (void)hipFree(c->d_ptw);
        if (c->d_label_map) (void)hipFree(c->d_label_map);
        if (c->d_col_path) (void)hipFree(c->d_col_path);
        if (c->d_col_leaf) (void)hipFree(c->d_col_leaf);
    }
    for (Workspace *w : {&c->ws_temp, &c->ws_counts, &c->ws_ovf, &c->ws_scan, &c->ws_rows, &c->ws_out, &c->ws_sort,
                         &c->ws_cls_off, &c->ws_cls_cols, &c->ws_class, &c->ws_sh_keys, &c->ws_sh_local, &c->ws_sh_cnt,
                         &c->ws_sh_sort, &c->ws_sh_tmp})
        if (w->buf) (void)hipFree(w->buf);
    free_host_pipe(c->pipe);
    if (c->d_scalars) (void)hipFree(c->d_scalars);
    if (c->h_scalars) (void)hipHostFree(c->h_scalars);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev_trav) (void)hipEventDestroy(c->ev_trav);
    if (c->ev_comp) (void)hipEventDestroy(c->ev_comp);
    if (c->s_compact) (void)hipStreamDestroy(c->s_compact);
    for (auto &pr : c->async_ev) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    destroy_fence(c->fence);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    Ctx *owner = c->image_owner;
    delete c;
    if (owner) {
        bool last;
        {
            std::lock_guard<std::mutex> lk(g_clone_mu);
            last = --owner->clones == 0 && owner->released;
        }
        if (last) release(owner);
    }
}

// a query context over src's image (mbrwt_ctx_clone)
static int clone_ctx(Ctx *src, Ctx **out) {
    *out = nullptr;
    Ctx *c = new (std::nothrow) Ctx();
    if (!c) return MBRWT_ERR_NOMEM;
    c->device = src->device;
    c->tree = src->tree;
    c->d_nodes = src->d_nodes;
    c->d_cnodes = src->d_cnodes;
    c->d_p2w = src->d_p2w;
    c->d_ptw = src->d_ptw;
    c->d_label_map = src->d_label_map;
    c->d_col_path = src->d_col_path;
    c->d_col_leaf = src->d_col_leaf;
    c->rows = src->rows;
    c->nodes_freed = src->nodes_freed;
    c->shard_rows = src->shard_rows;
    Ctx *owner = src->image_owner ? src->image_owner : src;
    c->image_owner = owner;
    {
        std::lock_guard<std::mutex> lk(g_clone_mu);
        ++owner->clones;
    }
    int rc = MBRWT_OK;
    if (hipSetDevice(c->device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
        rc = hip_fail(hipGetLastError(), "stream creation");
    if (!rc) rc = init_query_state(*c);
    for (size_t i = 0; !rc && i < src->shards.size(); ++i) {
        Ctx *sc = nullptr;
        rc = clone_ctx(src->shards[i], &sc);
        if (!rc) c->shards.push_back(sc);
    }
    if (rc) {
        release(c);
        return rc;
    }
    *out = c;
    return MBRWT_OK;
}

static int make_rows(Ctx &c, int layout);
// The layout a create call builds: NODES, ROWS or BOTH as set for the thread
// (mbrwt_set_build_option), else AUTO -- row records when the
// tree is within their limits and the image fits the device, the per-node
// images otherwise (make_rows, create_rows_ranged).
static int resolve_layout() { return build_layout(); }
constexpr int kNoLayoutHook = -1;

// layout: the finished context's layout (row records, make_rows);
// kNoLayoutHook for the sub-contexts of sharded / ranged builds
template <class Build>
static int create_common(int device, mbrwt_ctx **out, Build &&build, int layout = resolve_layout()) {
    if (!out) {
        set_error("null output pointer");
        return MBRWT_ERR_INVALID;
    }
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_error("no HIP device available");
        return MBRWT_ERR_DEVICE;
    }
    if (device < 0 || device >= ndev) {
        set_error("device index out of range");
        return MBRWT_ERR_INVALID;
    }
    Ctx *c = new (std::nothrow) Ctx();
    if (!c) return MBRWT_ERR_NOMEM;
    c->device = device;
    int rc = MBRWT_OK;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        rc = hip_fail(hipGetLastError(), "stream creation");
    }
    if (!rc) rc = build(*c);
    if (!rc) rc = upload_tables(*c);
    if (!rc && layout != kNoLayoutHook) rc = make_rows(*c, layout);
    if (rc) {
        release(c);
        return rc;
    }
    *out = reinterpret_cast<mbrwt_ctx *>(c);
    return MBRWT_OK;
}

static Ctx *C(mbrwt_ctx *p) { return reinterpret_cast<Ctx *>(p); }
static const Ctx *C(const mbrwt_ctx *p) { return reinterpret_cast<const Ctx *>(p); }

// A context over row shards (shards.hip): sub-contexts over the rows
// [k R, min(n, (k+1) R)), built in row order by build_shard(ctx, a, b).
template <class BuildShard>
static int create_sharded(int device, uint64_t num_rows, uint64_t num_columns, uint64_t R, mbrwt_ctx **out,
                          BuildShard &&build_shard, int layout) {
    return create_common(device, out, [&](Ctx &c) {
        c.tree.num_rows = num_rows;
        c.tree.num_columns = num_columns;
        c.shard_rows = R;
        for (uint64_t a = 0; a < num_rows; a += R) {
            const uint64_t b = std::min(num_rows, a + R);
            mbrwt_ctx *sub = nullptr;
            const int rc =
                create_common(device, &sub, [&](Ctx &sc) { return build_shard(sc, a, b); }, kNoLayoutHook);
            if (rc) return rc;
            Ctx *sc = C(sub);
            c.shards.push_back(sc);
            c.tree.num_relations += sc->tree.num_relations;
            c.tree.image_bytes += sc->tree.image_bytes;
            c.tree.num_nodes = sc->tree.num_nodes;
        }
        return MBRWT_OK;
    }, layout);
}

// Row records (rows.hip) of a finished node context -- unsharded, or over
// its row shards -- for layouts ROWS, BOTH and AUTO; ROWS and AUTO then drop
// the node images (and the shards).  AUTO keeps the node images instead when
// the tree is outside the row-record limits or the records do not fit.
constexpr uint64_t kRowsAlign = 360360;  // a multiple of every S <= 15
// rows per range of a ranged build: 1,073,512,440 (the build option
// MBRWT_BUILD_ROWS_RANGE, rounded up to a multiple of kRowsAlign, forces
// smaller ranges: a test hook)
static uint64_t rows_range_rows() {
    if (const uint64_t v = build_tuning().rows_range) return (v + kRowsAlign - 1) / kRowsAlign * kRowsAlign;
    return 2979ull * kRowsAlign;
}

static void drop_nodes(Ctx &c) {
    for (Ctx *sc : c.shards) release(sc);
    c.shards.clear();
    free_tree(c.tree);
    for (DevNode &d : c.tree.nodes) d.base = 0;
    c.tree.image_bytes = 0;
    c.nodes_freed = true;
}

static int make_rows(Ctx &c, int layout) {
    if (layout == LAYOUT_NODES) return MBRWT_OK;
    if (c.nodes_freed) return MBRWT_OK;
    if (c.tree.num_rows == 0) {
        if (layout == LAYOUT_AUTO) return MBRWT_OK;
        set_error("row records of a matrix without rows");
        return MBRWT_ERR_UNSUPPORTED;
    }
    const bool sharded = !c.shards.empty();
    RowsBuild *rb = rows_build_begin(c, c.tree.num_rows, sharded ? c.shard_rows : kRowsAlign, layout == LAYOUT_AUTO);
    if (!rb) return MBRWT_ERR_NOMEM;
    int rc = MBRWT_OK;
    if (!sharded) {
        rc = rows_build_range(rb, c, 0);
    } else {
        for (size_t k = 0; k < c.shards.size() && !rc; ++k) {
            rc = rows_build_range(rb, *c.shards[k], (uint64_t)k * c.shard_rows);
            if (!rc) (void)hipSetDevice(c.device);
        }
    }
    if (!rc) {
        rc = rows_build_finish(rb);
    } else {
        rows_build_abort(rb);
    }
    if (rc && layout == LAYOUT_AUTO && (rc == MBRWT_ERR_UNSUPPORTED || rc == MBRWT_ERR_NOMEM)) {
        (void)hipGetLastError();
        return MBRWT_OK;  // outside the row-record limits or too large: the per-node images answer
    }
    if (rc) return rc;
    if (layout != LAYOUT_BOTH) drop_nodes(c);
    return MBRWT_OK;
}

// Row records over many rows: the node image of one range of rows at a time
// (build_range(ctx, a, b), an ordinary context over rows [a, b)) is turned
// into its rows' records and released, so the device holds the records plus
// ONE range's node image.  The first range is small (kRowsAlign x 64 rows);
// it decides the record layout and measures the node image's bytes per row,
// from which every later range is sized to the memory left (at most
// rows_range_rows(); MBRWT_BUILD_ROWS_RANGE fixes the size: a test hook).
constexpr uint64_t kRowsFirstRange = 64 * kRowsAlign;
template <class BuildRange>
static int create_rows_ranged(int device, uint64_t num_rows, uint64_t num_columns, mbrwt_ctx **out, int layout,
                              BuildRange &&build_range) {
    return create_common(
        device, out,
        [&](Ctx &c) {
            c.tree.num_rows = num_rows;
            c.tree.num_columns = num_columns;
            const bool fixed = build_tuning().rows_range != 0;
            uint64_t R = fixed ? rows_range_rows() : std::min(rows_range_rows(), kRowsFirstRange);
            RowsBuild *rb = rows_build_begin(c, num_rows, kRowsAlign, layout == LAYOUT_AUTO);
            if (!rb) return (int)MBRWT_ERR_NOMEM;
            for (uint64_t a = 0, b = 0; a < num_rows; a = b) {
                b = std::min(num_rows, a + R);
                mbrwt_ctx *sub = nullptr;
                int rc = create_common(device, &sub, [&](Ctx &sc) { return build_range(sc, a, b); }, kNoLayoutHook);
                if (!rc) rc = rows_build_range(rb, *C(sub), a);
                if (!rc && !fixed && a == 0 && b < num_rows) {
                    // later ranges: what the first range's node image costs per
                    // row, into the memory its release leaves free less the
                    // records the later ranges will still allocate (the
                    // variable-length records: one allocation per range)
                    const double per_row = (double)C(sub)->tree.image_bytes / (double)(b - a);
                    size_t free_b = 0, total_b = 0;
                    (void)hipMemGetInfo(&free_b, &total_b);
                    const double avail = (double)free_b + (double)C(sub)->tree.image_bytes - 8.0 * (1ull << 30) -
                                         (double)rows_build_pending_bytes(rb, num_rows - b);
                    const double fit = per_row > 0 ? avail / (1.2 * per_row) : (double)rows_range_rows();
                    R = std::max<uint64_t>(kRowsAlign, std::min<uint64_t>(rows_range_rows(),
                                                                          (uint64_t)std::max(0.0, fit) / kRowsAlign *
                                                                              kRowsAlign));
                }
                if (!rc) {
                    const Tree &st = C(sub)->tree;
                    c.tree.num_relations += st.num_relations;
                    c.tree.num_nodes = st.num_nodes;
                    c.tree.max_arity = st.max_arity;
                    if (a == 0) {  // the shape (host tables only; no image)
                        c.tree.nodes = st.nodes;
                        c.tree.label_perm = st.label_perm;
                        c.tree.folded = st.folded;
                    }
                }
                if (sub) release(C(sub));
                (void)hipSetDevice(device);
                if (rc) {
                    rows_build_abort(rb);
                    return rc;
                }
            }
            const int rc = rows_build_finish(rb);
            if (rc) return rc;
            for (DevNode &d : c.tree.nodes) d.base = 0;
            c.nodes_freed = true;
            return (int)MBRWT_OK;
        },
        kNoLayoutHook);
}

// Layouts ROWS and AUTO over many rows build ranged: beyond kAutoRangedRows
// the whole node image and the records side by side may not fit (C3: 214 GB
// of node image + 160 GB of records).  AUTO falls back to the per-node
// images when the tree is outside the row-record limits or the records do
// not fit.  (MBRWT_BUILD_ROWS_RANGE: ranged beyond one such range, a test hook.)
constexpr uint64_t kAutoRangedRows = 1ull << 27;
static bool ranged_rows(int layout, uint64_t num_rows) {
    return (layout == LAYOUT_ROWS || layout == LAYOUT_AUTO) &&
           num_rows > std::min<uint64_t>(kAutoRangedRows, rows_range_rows());
}
static bool auto_fallback(int layout, int rc) {
    if (layout != LAYOUT_AUTO || (rc != MBRWT_ERR_UNSUPPORTED && rc != MBRWT_ERR_NOMEM)) return false;
    (void)hipGetLastError();
    return true;
}

// the synthetic law over row shards: shard k draws node u's masks at the
// positions after those of shards 0..k-1 (SynthShard, synth.hip)
static int create_synthetic_any(const mbrwt_synth_desc &desc, const mbrwt_shape_desc *shape, int device,
                                mbrwt_ctx **out) {
    int layout = resolve_layout();
    if (ranged_rows(layout, desc.num_rows) && desc.num_columns) {
        SynthShard st;
        std::vector<uint64_t> lens;
        st.len_out = &lens;
        const int rc =
            create_rows_ranged(device, desc.num_rows, desc.num_columns, out, layout, [&](Ctx &sc, uint64_t a, uint64_t b) {
            mbrwt_synth_desc d = desc;
            d.num_rows = b - a;
            st.row0 = a;
            const int rc = build_synthetic(d, shape, device, sc.tree, sc.stream, &st);
            if (rc) return rc;
            if (st.pos0.size() < lens.size()) st.pos0.resize(lens.size(), 0);
            for (size_t u = 0; u < lens.size(); ++u) st.pos0[u] += lens[u];
            return (int)MBRWT_OK;
        });
        if (!auto_fallback(layout, rc)) return rc;
        layout = LAYOUT_NODES;
    }
    const uint64_t R = desc.num_columns ? shard_rows_for(desc.num_rows) : 0;
    if (!R)
        return create_common(
            device, out, [&](Ctx &c) { return build_synthetic(desc, shape, device, c.tree, c.stream); }, layout);
    SynthShard st;
    std::vector<uint64_t> lens;
    st.len_out = &lens;
    return create_sharded(
        device, desc.num_rows, desc.num_columns, R, out,
        [&](Ctx &sc, uint64_t a, uint64_t b) {
            mbrwt_synth_desc d = desc;
            d.num_rows = b - a;
            st.row0 = a;
            const int rc = build_synthetic(d, shape, device, sc.tree, sc.stream, &st);
            if (rc) return rc;
            if (st.pos0.size() < lens.size()) st.pos0.resize(lens.size(), 0);
            for (size_t u = 0; u < lens.size(); ++u) st.pos0[u] += lens[u];
            return (int)MBRWT_OK;
        },
        layout);
}

}  // namespace mbrwt

using namespace mbrwt;

extern "C" {

int mbrwt_create(const mbrwt_tree_desc *desc, int device, mbrwt_ctx **out) {
    if (!desc) {
        set_error("null tree description");
        return MBRWT_ERR_INVALID;
    }
    try {
        int layout = resolve_layout();
        if (ranged_rows(layout, desc->num_rows) && desc->num_nodes) {
            const int rc = create_rows_ranged(device, desc->num_rows, desc->num_columns, out, layout,
                                              [&](Ctx &sc, uint64_t a, uint64_t b) {
                                                  SlicedDesc sd;
                                                  const int rc = slice_desc(*desc, a, b, sd);
                                                  return rc ? rc : build_from_desc(sd.desc, device, sc.tree);
                                              });
            if (!auto_fallback(layout, rc)) return rc;
            layout = LAYOUT_NODES;
        }
        const uint64_t R = desc->num_nodes ? shard_rows_for(desc->num_rows) : 0;
        if (R) {  // rows >= 2^32: every shard is built from the description's slice
            return create_sharded(
                device, desc->num_rows, desc->num_columns, R, out,
                [&](Ctx &sc, uint64_t a, uint64_t b) {
                    SlicedDesc sd;
                    const int rc = slice_desc(*desc, a, b, sd);
                    return rc ? rc : build_from_desc(sd.desc, device, sc.tree);
                },
                layout);
        }
        return create_common(device, out, [&](Ctx &c) { return build_from_desc(*desc, device, c.tree); }, layout);
    } catch (const std::bad_alloc &) {
        set_error("host allocation failed");
        return MBRWT_ERR_NOMEM;
    } catch (...) {
        set_error("unexpected exception in mbrwt_create");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_create_synthetic_shaped(const mbrwt_synth_desc *desc, const mbrwt_shape_desc *shape, int device,
                                  mbrwt_ctx **out) {
    if (!desc || !shape) {
        set_error("null synthetic or shape description");
        return MBRWT_ERR_INVALID;
    }
    try {
        return create_synthetic_any(*desc, shape, device, out);
    } catch (const std::bad_alloc &) {
        set_error("host allocation failed");
        return MBRWT_ERR_NOMEM;
    } catch (...) {
        set_error("unexpected exception in mbrwt_create_synthetic_shaped");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_create_synthetic(const mbrwt_synth_desc *desc, int device, mbrwt_ctx **out) {
    if (!desc) {
        set_error("null synthetic description");
        return MBRWT_ERR_INVALID;
    }
    try {
        return create_synthetic_any(*desc, nullptr, device, out);
    } catch (const std::bad_alloc &) {
        set_error("host allocation failed");
        return MBRWT_ERR_NOMEM;
    } catch (...) {
        set_error("unexpected exception in mbrwt_create_synthetic");
        return MBRWT_ERR_INVALID;
    }
}

// rows >= 2^32 (Row = uint64_t, binary_matrix.hpp:11): the device builders
// produce the tree description on a temporary stream and hand it to
// mbrwt_create, which builds row shards (or row-record ranges) from it
static int create_via_desc(int device, mbrwt_ctx **out,
                           const std::function<int(hipStream_t, const DescSink &)> &build) {
    if (!out) {
        set_error("null output pointer");
        return MBRWT_ERR_INVALID;
    }
    MBRWT_HIP(hipSetDevice(device));
    hipStream_t s = nullptr;
    MBRWT_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int rc = build(s, [&](const mbrwt_tree_desc &d) { return mbrwt_create(&d, device, out); });
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
    return rc;
}

int mbrwt_create_from_columns(const mbrwt_columns_desc *desc, int device, mbrwt_ctx **out) {
    if (!desc) {
        set_error("null columns description");
        return MBRWT_ERR_INVALID;
    }
    try {
        if (desc->num_rows > kMaxRows)
            return create_via_desc(device, out, [&](hipStream_t s, const DescSink &emit) {
                return desc_from_columns(*desc, device, s, 0, emit);
            });
        return create_common(device, out,
                             [&](Ctx &c) { return build_from_columns(*desc, device, c.tree, c.stream); });
    } catch (const std::bad_alloc &) {
        set_error("host allocation failed");
        return MBRWT_ERR_NOMEM;
    } catch (...) {
        set_error("unexpected exception in mbrwt_create_from_columns");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_create_from_columns_relaxed(const mbrwt_columns_desc *desc, uint64_t relax_max_arity, int device,
                                      mbrwt_ctx **out) {
    if (!desc) {
        set_error("null columns description");
        return MBRWT_ERR_INVALID;
    }
    try {
        if (desc->num_rows > kMaxRows)
            return create_via_desc(device, out, [&](hipStream_t s, const DescSink &emit) {
                return desc_from_columns(*desc, device, s, relax_max_arity, emit);
            });
        return create_common(device, out, [&](Ctx &c) {
            return build_from_columns(*desc, device, c.tree, c.stream, relax_max_arity);
        });
    } catch (const std::bad_alloc &) {
        set_error("host allocation failed");
        return MBRWT_ERR_NOMEM;
    } catch (...) {
        set_error("unexpected exception in mbrwt_create_from_columns_relaxed");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_create_relaxed(const mbrwt_tree_desc *desc, uint64_t max_arity, int device, mbrwt_ctx **out) {
    if (!desc) {
        set_error("null tree description");
        return MBRWT_ERR_INVALID;
    }
    try {
        if (desc->num_rows > kMaxRows)
            return create_via_desc(device, out, [&](hipStream_t s, const DescSink &emit) {
                return relaxed_desc(*desc, max_arity, device, s, emit);
            });
        return create_common(device, out, [&](Ctx &c) {
            return build_relaxed_from_desc(*desc, max_arity, device, c.tree, c.stream);
        });
    } catch (const std::bad_alloc &) {
        set_error("host allocation failed");
        return MBRWT_ERR_NOMEM;
    } catch (...) {
        set_error("unexpected exception in mbrwt_create_relaxed");
        return MBRWT_ERR_INVALID;
    }
}

void mbrwt_destroy(mbrwt_ctx *ctx) { release(C(ctx)); }

int mbrwt_ctx_clone(mbrwt_ctx *src, mbrwt_ctx **out) {
    if (!src || !out) {
        set_error("null context or output pointer");
        return MBRWT_ERR_INVALID;
    }
    Ctx *c = nullptr;
    const int rc = clone_ctx(C(src), &c);
    *out = reinterpret_cast<mbrwt_ctx *>(c);
    return rc;
}

uint64_t mbrwt_num_rows(const mbrwt_ctx *ctx) { return ctx ? C(ctx)->tree.num_rows : 0; }
uint64_t mbrwt_num_columns(const mbrwt_ctx *ctx) { return ctx ? C(ctx)->tree.num_columns : 0; }
uint64_t mbrwt_num_relations(const mbrwt_ctx *ctx) { return ctx ? C(ctx)->tree.num_relations : 0; }
uint64_t mbrwt_num_nodes(const mbrwt_ctx *ctx) { return ctx ? C(ctx)->tree.num_nodes : 0; }
uint64_t mbrwt_device_bytes(const mbrwt_ctx *ctx) { return ctx ? C(ctx)->tree.image_bytes + C(ctx)->rows.bytes : 0; }

int mbrwt_set_build_option(int option, int64_t value) {
    BuildTuning &t = build_tuning();
    switch (option) {
    case MBRWT_BUILD_ROWS_VAR:
        if (value < -1 || value > 1) break;
        t.rows_var = (int)value;
        return MBRWT_OK;
    case MBRWT_BUILD_VAR_LANES:
        if (value < 0 || value > 16 || (value & (value - 1))) break;
        t.var_lanes = (uint32_t)value;
        return MBRWT_OK;
    case MBRWT_BUILD_ROWS_BLOCK: {
        const int64_t Bv = value >> 8, Sv = value & 0xFF;
        if (value != 0 && !((Bv == 64 && Sv >= 1 && Sv <= 8) || (Bv == 128 && Sv >= 1 && Sv <= 15))) break;
        t.rows_block = (uint32_t)value;
        return MBRWT_OK;
    }
    case MBRWT_BUILD_ROWS_RANGE:
        if (value < 0) break;
        t.rows_range = (uint64_t)value;
        return MBRWT_OK;
    case MBRWT_BUILD_NODE_KINDS:
        if (value < 0 || value > MBRWT_KIND_ALL) break;
        t.node_kinds = (uint32_t)value;
        return MBRWT_OK;
    case MBRWT_BUILD_SHARD_ROWS:
        if (value < 0) break;
        t.shard_rows = (uint64_t)value;
        return MBRWT_OK;
    case MBRWT_BUILD_ROWS_WGS_PER_CU:
        if (value < 0 || value > 32) break;
        t.rows_wgs_per_cu = (uint32_t)value;
        return MBRWT_OK;
    case MBRWT_BUILD_ROWS_CLASSES:
        if (value < -1 || value > 1) break;
        t.rows_classes = (int)value;
        return MBRWT_OK;
    case MBRWT_BUILD_ROWS_CODE:
        if (value < 0 || value > 3) break;
        t.rows_code = (int)value;
        return MBRWT_OK;
    default:
        break;
    }
    if (option >= MBRWT_BUILD_ROWS_VAR && option <= MBRWT_BUILD_ROWS_CODE) {
        set_error("build option value out of range");
        return MBRWT_ERR_INVALID;
    }
    if (option == MBRWT_BUILD_PARTITIONER &&
        (value == MBRWT_PARTITIONER_BASIC || value == MBRWT_PARTITIONER_GREEDY)) {
        set_build_partitioner((int)value);
        return MBRWT_OK;
    }
    if (option == MBRWT_BUILD_ROWS_FOOTPRINT && (value == MBRWT_ROWS_FAST || value == MBRWT_ROWS_COMPACT)) {
        set_rows_footprint((int)value);
        return MBRWT_OK;
    }
    if (option != MBRWT_BUILD_LAYOUT || value < MBRWT_LAYOUT_AUTO || value > MBRWT_LAYOUT_BOTH) {
        set_error("unknown build option or value");
        return MBRWT_ERR_INVALID;
    }
    set_build_layout((int)value);
    return MBRWT_OK;
}

int mbrwt_get_build_option(int option, int64_t *value) {
    if (!value || option < MBRWT_BUILD_LAYOUT || option > MBRWT_BUILD_ROWS_CODE) {
        set_error("unknown build option or null output");
        return MBRWT_ERR_INVALID;
    }
    const BuildTuning &t = build_tuning();
    switch (option) {
    case MBRWT_BUILD_LAYOUT: *value = thread_build_layout(); break;
    case MBRWT_BUILD_PARTITIONER: *value = build_partitioner(); break;
    case MBRWT_BUILD_ROWS_FOOTPRINT: *value = rows_footprint(); break;
    case MBRWT_BUILD_ROWS_VAR: *value = t.rows_var; break;
    case MBRWT_BUILD_VAR_LANES: *value = t.var_lanes; break;
    case MBRWT_BUILD_ROWS_BLOCK: *value = t.rows_block; break;
    case MBRWT_BUILD_ROWS_RANGE: *value = (int64_t)t.rows_range; break;
    case MBRWT_BUILD_NODE_KINDS: *value = t.node_kinds; break;
    case MBRWT_BUILD_SHARD_ROWS: *value = (int64_t)t.shard_rows; break;
    case MBRWT_BUILD_ROWS_WGS_PER_CU: *value = t.rows_wgs_per_cu; break;
    case MBRWT_BUILD_ROWS_CLASSES: *value = t.rows_classes; break;
    default: *value = t.rows_code; break;
    }
    return MBRWT_OK;
}

int mbrwt_layout(const mbrwt_ctx *ctx) {
    if (!ctx) return 0;
    const Ctx &c = *C(ctx);
    return !c.rows.ready ? MBRWT_LAYOUT_NODES : c.nodes_freed ? MBRWT_LAYOUT_ROWS : MBRWT_LAYOUT_BOTH;
}

int mbrwt_rows_stats(const mbrwt_ctx *ctx, uint64_t out[8]) {
    if (!ctx || !out) return MBRWT_ERR_INVALID;
    const RowsImage &r = C(ctx)->rows;
    if (!r.ready) {
        set_error("context has no row records");
        return MBRWT_ERR_UNSUPPORTED;
    }
    out[0] = r.var ? 0 : r.B;  // 0: variable-length records (rows_var.hip)
    out[1] = r.var ? 13 : r.S;
    out[2] = r.var ? (C(ctx)->tree.num_rows + 12) / 13 * 64 : r.num_blocks * r.B;
    out[3] = r.spill_bytes;
    out[4] = r.record_bytes;
    out[5] = r.spilled_rows;
    out[6] = r.long_rows;
    out[7] = r.height | (uint64_t)r.uni << 32 | (uint64_t)(r.nib ? 1 : 0) << 40 | (uint64_t)(r.term ? 1 : 0) << 41;
    return MBRWT_OK;
}
int mbrwt_rows_classes(const mbrwt_ctx *ctx, uint64_t out[4]) {
    if (!ctx || !out) return MBRWT_ERR_INVALID;
    const RowsImage &r = C(ctx)->rows;
    if (!r.ready) {
        set_error("context has no row records");
        return MBRWT_ERR_UNSUPPORTED;
    }
    out[0] = r.num_classes;
    out[1] = r.class_bits;
    out[2] = r.class_index_bytes;
    out[3] = r.class_sample_distinct;
    return MBRWT_OK;
}
int mbrwt_device(const mbrwt_ctx *ctx) { return ctx ? C(ctx)->device : -1; }
uint64_t mbrwt_num_shards(const mbrwt_ctx *ctx) { return ctx ? std::max<uint64_t>(1, C(ctx)->shards.size()) : 0; }

int mbrwt_get_rows_device(mbrwt_ctx *ctx, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets, uint32_t *d_cols,
                          uint64_t cols_cap, uint64_t *cols_needed, void *stream) {
    if (!ctx || (n && (!d_rows || !d_offsets)) || (!n && !d_offsets)) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    WsFence fence_(c.fence, reinterpret_cast<hipStream_t>(stream));
    try {
        if (hipSetDevice(c.device) != hipSuccess) return hip_fail(hipGetLastError(), "hipSetDevice");
        return run_get_rows(c, d_rows, n, d_offsets, d_cols, d_cols ? cols_cap : 0, cols_needed,
                            reinterpret_cast<hipStream_t>(stream));
    } catch (...) {
        set_error("unexpected exception in mbrwt_get_rows_device");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_get_rows_device_async(mbrwt_ctx *ctx, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets,
                                uint32_t *d_cols, uint64_t cols_cap, uint64_t *d_status, void *stream) {
    if (!ctx || !d_status || (n && (!d_rows || !d_offsets)) || (!n && !d_offsets)) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    Ctx &c = *C(ctx);
    const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    std::lock_guard<std::mutex> lk(c.mu);
    WsFence fence_(c.fence, s);
    try {
        if (hipSetDevice(c.device) != hipSuccess) return hip_fail(hipGetLastError(), "hipSetDevice");
        if (c.rows.ready && c.kernel_variant == 0 && n > 0)
            return rows_get_rows(c, d_rows, n, d_offsets, d_cols, d_cols ? cols_cap : 0, nullptr, s, d_status);
        // other images: the synchronous call, then its status on the stream
        uint64_t need = 0;
        const int rc = run_get_rows(c, d_rows, n, d_offsets, d_cols, d_cols ? cols_cap : 0, &need, s);
        if (rc != MBRWT_OK && rc != MBRWT_ERR_CAPACITY && rc != MBRWT_ERR_RANGE) return rc;
        return rows_set_status(d_status, need, rc, s);
    } catch (...) {
        set_error("unexpected exception in mbrwt_get_rows_device_async");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_get_rows(mbrwt_ctx *ctx, const uint64_t *rows, uint64_t n, uint64_t *offsets, uint32_t *cols,
                   uint64_t cols_cap, uint64_t *cols_needed) {
    if (!ctx || !offsets || (n && !rows)) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    WsFence fence_(c.fence, c.stream);
    try {
        MBRWT_HIP(hipSetDevice(c.device));
        // chunks of the batch pipelined over PCIe (hostpipe.cpp)
        return host_get_rows(c, rows, n, offsets, cols, cols ? cols_cap : 0, cols_needed);
    } catch (...) {
        set_error("unexpected exception in mbrwt_get_rows");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_get_column_device(mbrwt_ctx *ctx, uint64_t column, uint64_t *d_rows, uint64_t rows_cap,
                            uint64_t *rows_needed, void *stream) {
    if (!ctx) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    WsFence fence_(c.fence, reinterpret_cast<hipStream_t>(stream));
    try {
        MBRWT_HIP(hipSetDevice(c.device));
        return run_get_column(c, column, d_rows, d_rows ? rows_cap : 0, rows_needed,
                              reinterpret_cast<hipStream_t>(stream));
    } catch (...) {
        set_error("unexpected exception in mbrwt_get_column_device");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_get_column(mbrwt_ctx *ctx, uint64_t column, uint64_t *rows, uint64_t rows_cap, uint64_t *rows_needed) {
    if (!ctx) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    WsFence fence_(c.fence, c.stream);
    try {
        MBRWT_HIP(hipSetDevice(c.device));
        int rc;
        uint64_t needed = 0;
        // the column's size is known after the first (counting) phase
        if ((rc = ensure(c.ws_out, std::max<uint64_t>(rows_cap, 1) * sizeof(uint64_t)))) return rc;
        rc = run_get_column(c, column, reinterpret_cast<uint64_t *>(c.ws_out.buf), rows ? rows_cap : 0, &needed,
                            c.stream);
        if (rows_needed) *rows_needed = needed;
        if (rc) return rc;
        if (needed)
            MBRWT_HIP(hipMemcpyAsync(rows, c.ws_out.buf, needed * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
        MBRWT_HIP(hipStreamSynchronize(c.stream));
        return MBRWT_OK;
    } catch (...) {
        set_error("unexpected exception in mbrwt_get_column");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_get_batch_device(mbrwt_ctx *ctx, const uint64_t *d_rows, const uint64_t *d_cols, uint64_t n,
                           uint8_t *d_out, void *stream) {
    if (!ctx || (n && (!d_rows || !d_cols || !d_out))) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    WsFence fence_(c.fence, reinterpret_cast<hipStream_t>(stream));
    MBRWT_HIP(hipSetDevice(c.device));
    return run_get_batch(c, d_rows, d_cols, n, d_out, reinterpret_cast<hipStream_t>(stream));
}

int mbrwt_get_batch(mbrwt_ctx *ctx, const uint64_t *rows, const uint64_t *cols, uint64_t n, uint8_t *out) {
    if (!ctx || (n && (!rows || !cols || !out))) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    WsFence fence_(c.fence, c.stream);
    MBRWT_HIP(hipSetDevice(c.device));
    if (!n) return MBRWT_OK;
    int rc;
    if ((rc = ensure(c.ws_rows, n * sizeof(uint64_t) * 2 + n))) return rc;
    uint64_t *d_r = reinterpret_cast<uint64_t *>(c.ws_rows.buf);
    uint64_t *d_c = d_r + n;
    uint8_t *d_o = reinterpret_cast<uint8_t *>(d_c + n);
    MBRWT_HIP(hipMemcpyAsync(d_r, rows, n * 8, hipMemcpyHostToDevice, c.stream));
    MBRWT_HIP(hipMemcpyAsync(d_c, cols, n * 8, hipMemcpyHostToDevice, c.stream));
    rc = run_get_batch(c, d_r, d_c, n, d_o, c.stream);
    if (rc) return rc;
    MBRWT_HIP(hipMemcpyAsync(out, d_o, n, hipMemcpyDeviceToHost, c.stream));
    MBRWT_HIP(hipStreamSynchronize(c.stream));
    return MBRWT_OK;
}

int mbrwt_count_labels_device(mbrwt_ctx *ctx, const uint64_t *d_rows, uint64_t n, uint64_t *d_counts,
                              void *stream) {
    if (!ctx || (n && !d_rows) || !d_counts) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    WsFence fence_(c.fence, reinterpret_cast<hipStream_t>(stream));
    MBRWT_HIP(hipSetDevice(c.device));
    return run_count_labels(c, d_rows, n, d_counts, reinterpret_cast<hipStream_t>(stream));
}

int mbrwt_get_labels_batch_device(mbrwt_ctx *ctx, const uint64_t *d_rows, uint64_t n_rows,
                                  const uint64_t *d_read_offsets, uint64_t n_reads, double presence_ratio,
                                  uint64_t *d_label_offsets, uint32_t *d_labels, uint64_t labels_cap,
                                  uint64_t *labels_needed, void *stream) {
    if (!ctx || (n_rows && !d_rows) || !d_read_offsets || !d_label_offsets) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    WsFence fence_(c.fence, reinterpret_cast<hipStream_t>(stream));
    try {
        MBRWT_HIP(hipSetDevice(c.device));
        return run_get_labels_batch(c, d_rows, n_rows, d_read_offsets, n_reads, presence_ratio, d_label_offsets,
                                    d_labels, d_labels ? labels_cap : 0, labels_needed,
                                    reinterpret_cast<hipStream_t>(stream));
    } catch (...) {
        set_error("unexpected exception in mbrwt_get_labels_batch_device");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_get_labels_batch(mbrwt_ctx *ctx, const uint64_t *rows, uint64_t n_rows, const uint64_t *read_offsets,
                           uint64_t n_reads, double presence_ratio, uint64_t *label_offsets, uint32_t *labels,
                           uint64_t labels_cap, uint64_t *labels_needed) {
    if (!ctx || (n_rows && !rows) || !read_offsets || !label_offsets) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    WsFence fence_(c.fence, c.stream);
    try {
        MBRWT_HIP(hipSetDevice(c.device));
        int rc;
        // rows | read offsets | label offsets, one host-path workspace
        if ((rc = ensure(c.ws_rows, (n_rows + 2 * (n_reads + 1)) * sizeof(uint64_t)))) return rc;
        uint64_t *d_rows = reinterpret_cast<uint64_t *>(c.ws_rows.buf);
        uint64_t *d_roff = d_rows + n_rows;
        uint64_t *d_loff = d_roff + n_reads + 1;
        if (n_rows) MBRWT_HIP(hipMemcpyAsync(d_rows, rows, n_rows * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream));
        MBRWT_HIP(hipMemcpyAsync(d_roff, read_offsets, (n_reads + 1) * sizeof(uint64_t), hipMemcpyHostToDevice,
                                 c.stream));
        if ((rc = ensure(c.ws_out, std::max<uint64_t>(labels_cap, 1) * sizeof(uint32_t)))) return rc;
        uint64_t needed = 0;
        rc = run_get_labels_batch(c, d_rows, n_rows, d_roff, n_reads, presence_ratio, d_loff,
                                  reinterpret_cast<uint32_t *>(c.ws_out.buf), labels ? labels_cap : 0, &needed,
                                  c.stream);
        if (labels_needed) *labels_needed = needed;
        if (rc) return rc;
        MBRWT_HIP(hipMemcpyAsync(label_offsets, d_loff, (n_reads + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                 c.stream));
        if (needed)
            MBRWT_HIP(hipMemcpyAsync(labels, c.ws_out.buf, needed * sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
        MBRWT_HIP(hipStreamSynchronize(c.stream));
        return MBRWT_OK;
    } catch (...) {
        set_error("unexpected exception in mbrwt_get_labels_batch");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_get_top_labels_batch_device(mbrwt_ctx *ctx, const uint64_t *d_rows, uint64_t n_rows,
                                      const uint64_t *d_read_offsets, uint64_t n_reads, uint64_t num_top,
                                      uint64_t *d_label_offsets, uint32_t *d_labels, uint64_t *d_counts,
                                      uint64_t labels_cap, uint64_t *labels_needed, void *stream) {
    if (!ctx || (n_rows && !d_rows) || !d_read_offsets || !d_label_offsets) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    WsFence fence_(c.fence, reinterpret_cast<hipStream_t>(stream));
    try {
        MBRWT_HIP(hipSetDevice(c.device));
        const bool out = d_labels && d_counts;
        return run_get_top_labels_batch(c, d_rows, n_rows, d_read_offsets, n_reads, num_top, d_label_offsets,
                                        d_labels, d_counts, out ? labels_cap : 0, labels_needed,
                                        reinterpret_cast<hipStream_t>(stream));
    } catch (...) {
        set_error("unexpected exception in mbrwt_get_top_labels_batch_device");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_get_top_labels_batch(mbrwt_ctx *ctx, const uint64_t *rows, uint64_t n_rows, const uint64_t *read_offsets,
                               uint64_t n_reads, uint64_t num_top, uint64_t *label_offsets, uint32_t *labels,
                               uint64_t *counts, uint64_t labels_cap, uint64_t *labels_needed) {
    if (!ctx || (n_rows && !rows) || !read_offsets || !label_offsets) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    WsFence fence_(c.fence, c.stream);
    try {
        MBRWT_HIP(hipSetDevice(c.device));
        int rc;
        if ((rc = ensure(c.ws_rows, (n_rows + 2 * (n_reads + 1)) * sizeof(uint64_t)))) return rc;
        uint64_t *d_rows = reinterpret_cast<uint64_t *>(c.ws_rows.buf);
        uint64_t *d_roff = d_rows + n_rows;
        uint64_t *d_loff = d_roff + n_reads + 1;
        if (n_rows) MBRWT_HIP(hipMemcpyAsync(d_rows, rows, n_rows * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream));
        MBRWT_HIP(hipMemcpyAsync(d_roff, read_offsets, (n_reads + 1) * sizeof(uint64_t), hipMemcpyHostToDevice,
                                 c.stream));
        // labels (u32) then counts (u64, 8-byte aligned) in the host-path output workspace
        const uint64_t lab_words = (std::max<uint64_t>(labels_cap, 1) + 1) & ~1ull;
        if ((rc = ensure(c.ws_out, lab_words * sizeof(uint32_t) + std::max<uint64_t>(labels_cap, 1) * 8))) return rc;
        uint32_t *d_lab = reinterpret_cast<uint32_t *>(c.ws_out.buf);
        uint64_t *d_cnt = reinterpret_cast<uint64_t *>(d_lab + lab_words);
        uint64_t needed = 0;
        const bool out = labels && counts;
        rc = run_get_top_labels_batch(c, d_rows, n_rows, d_roff, n_reads, num_top, d_loff, d_lab, d_cnt,
                                      out ? labels_cap : 0, &needed, c.stream);
        if (labels_needed) *labels_needed = needed;
        if (rc) return rc;
        MBRWT_HIP(hipMemcpyAsync(label_offsets, d_loff, (n_reads + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                 c.stream));
        if (needed) {
            MBRWT_HIP(hipMemcpyAsync(labels, d_lab, needed * sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
            MBRWT_HIP(hipMemcpyAsync(counts, d_cnt, needed * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
        }
        MBRWT_HIP(hipStreamSynchronize(c.stream));
        return MBRWT_OK;
    } catch (...) {
        set_error("unexpected exception in mbrwt_get_top_labels_batch");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_count_work_device(mbrwt_ctx *ctx, const uint64_t *d_rows, uint64_t n, uint64_t *sum_visits,
                            uint64_t *sum_labels, void *stream) {
    if (!ctx || (n && !d_rows)) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    WsFence fence_(c.fence, reinterpret_cast<hipStream_t>(stream));
    MBRWT_HIP(hipSetDevice(c.device));
    return run_count_work(c, d_rows, n, sum_visits, sum_labels, reinterpret_cast<hipStream_t>(stream));
}

static int apply_option(Ctx &c, int option, int64_t value) {
    for (Ctx *sc : c.shards)
        if (const int rc = apply_option(*sc, option, value)) return rc;
    switch (option) {
    case MBRWT_OPT_TIMING:
        c.timing = value != 0;
        return MBRWT_OK;
    case MBRWT_OPT_SLOT_LABELS:
        if (value < 0 || value > 4096) return MBRWT_ERR_INVALID;
        c.slot_labels = (uint32_t)value;
        return MBRWT_OK;
    case MBRWT_OPT_ROWS_WALK:
        if (value != 0 && value != 3 && value != 4 && value != 6 && value != 7) return MBRWT_ERR_INVALID;
        c.rows_walk = (int)value;
        return MBRWT_OK;
    case MBRWT_OPT_TEST_FAIL_CHUNK:
        c.test_fail_chunk = value < 0 ? -1 : value;
        return MBRWT_OK;
    case MBRWT_OPT_COMPACT_CUS: {
        if (value < 0 || value > 31) return MBRWT_ERR_INVALID;
        if ((uint32_t)value == c.compact_cus) return MBRWT_OK;
        MBRWT_HIP(hipSetDevice(c.device));
        if (c.s_compact) {
            MBRWT_HIP(hipStreamSynchronize(c.s_compact));
            MBRWT_HIP(hipStreamDestroy(c.s_compact));
            c.s_compact = nullptr;
        }
        c.compact_cus = 0;
        if (value == 0) return MBRWT_OK;
        // CU k is in the mask when k % 32 < value: the same share of every
        // XCD whether the logical CU ids run across the XCDs or within them
        int cus = 0;
        MBRWT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c.device));
        std::vector<uint32_t> mask((std::max(cus, 1) + 31) / 32, 0u);
        for (int k = 0; k < cus; ++k)
            if ((uint32_t)(k % 32) < (uint32_t)value) mask[k / 32] |= 1u << (k % 32);
        MBRWT_HIP(hipExtStreamCreateWithCUMask(&c.s_compact, (uint32_t)mask.size(), mask.data()));
        if (!c.ev_trav) MBRWT_HIP(hipEventCreateWithFlags(&c.ev_trav, hipEventDisableTiming));
        if (!c.ev_comp) MBRWT_HIP(hipEventCreateWithFlags(&c.ev_comp, hipEventDisableTiming));
        c.compact_cus = (uint32_t)value;
        return MBRWT_OK;
    }
    case MBRWT_OPT_KERNEL:
        if (!(value >= 0 && value <= 6) && value != 10 && !(value >= 17 && value <= 20) && !(value >= 24 && value <= 30))
            return MBRWT_ERR_INVALID;
        // the release library dispatches the default families only: 0, and 1
        // (the lane-per-row general kernel); the measured r02-r04 variants
        // were retired (r06; their results are in profiles/r02..r04)
        if (value > 1) {
            set_error("kernel variant retired: only 0 and 1 are dispatched");
            return MBRWT_ERR_UNSUPPORTED;
        }
        if (value != 0 && c.nodes_freed) {  // (a variant would fail at query time)
            set_error("kernel variants run on the node image: build with layout NODES or BOTH");
            return MBRWT_ERR_UNSUPPORTED;
        }
        c.kernel_variant = (int)value;
        return MBRWT_OK;
    default:
        set_error("unknown option");
        return MBRWT_ERR_INVALID;
    }
}

int mbrwt_set_option(mbrwt_ctx *ctx, int option, int64_t value) {
    if (!ctx) return MBRWT_ERR_INVALID;
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    return apply_option(c, option, value);
}

int mbrwt_take_timing(mbrwt_ctx *ctx, double *kernel_ms, uint64_t *launches) {
    if (!ctx) return MBRWT_ERR_INVALID;
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    for (size_t i = 0; i < c.async_used; ++i) {  // asynchronous calls' event pairs
        float ms = 0;
        MBRWT_HIP(hipEventSynchronize(c.async_ev[i].second));
        MBRWT_HIP(hipEventElapsedTime(&ms, c.async_ev[i].first, c.async_ev[i].second));
        c.timing_ms += ms;
        c.timing_launches += 1;
    }
    c.async_used = 0;
    for (Ctx *sc : c.shards) {  // a sharded context's kernels run on its shards
        c.timing_ms += sc->timing_ms;
        c.timing_launches += sc->timing_launches;
        sc->timing_ms = 0;
        sc->timing_launches = 0;
    }
    if (kernel_ms) *kernel_ms = c.timing_ms;
    if (launches) *launches = c.timing_launches;
    c.timing_ms = 0;
    c.timing_launches = 0;
    return MBRWT_OK;
}

const char *mbrwt_strerror(int status) {
    switch (status) {
    case MBRWT_OK: return "ok";
    case MBRWT_ERR_INVALID: return "invalid argument";
    case MBRWT_ERR_RANGE: return "row or column out of range";
    case MBRWT_ERR_CAPACITY: return "output capacity too small";
    case MBRWT_ERR_UNSUPPORTED: return "unsupported tree shape";
    case MBRWT_ERR_DEVICE: return "HIP device error";
    case MBRWT_ERR_NOMEM: return "out of memory";
    default: return "unknown status";
    }
}

const char *mbrwt_last_error_message(void) { return g_last_error.c_str(); }

const char *mbrwt_traverse_kernel(mbrwt_ctx *ctx) {
    if (!ctx) return "";
    Ctx &c = *C(ctx);
    std::lock_guard<std::mutex> lk(c.mu);
    return traverse_kernel_name(c.shards.empty() ? c : *c.shards[0]);
}

}  // extern "C"

// mbrwt_internal.hpp -- device image format and context of libmbrwt.
//
// Device image of a BRWT (DESIGN.md "Data layout in HBM"):
//   * dnode 0 is a virtual super-root with one child, the BRWT root; dnode
//     u+1 is tree node u (BFS numbering of mbrwt_tree_desc).  Visiting the
//     super-root at position `row` reads the root's index bit and rank, so
//     get_row(row) is one uniform descent (BRWT.cpp:30 + :43).
//   * An internal node u does not store its own index column; it stores the
//     columns of ALL its children interleaved ("sibling-interleaved"): every
//     child of u is probed at the same index j = rank1(u, i) - 1
//     (BRWT.cpp:43-51), so one block read answers every child's
//     operator[] and rank1 at j:
//       KIND_PLANE : per 32-position block, for each child c an 8-byte
//                    {u32 rank of child c before the block, u32 bits of child
//                    c in the block}; block stride = pow2ceil(8 * arity).
//       KIND_MASK* : (all children are leaves) one arity-bit mask per position,
//                    1/2/4/8 bytes wide; leaves need no rank.
//   * Leaves have no image; their global column (RangePartition::get composed
//     along the path, utils.cpp:689-691) is in DevNode::label.
//   * Root folding: when the root's index column is at least half full, the
//     super-root stores the root's CHILDREN interleaved over row positions
//     (a child bit is 0 where the root bit is 0), so get_row starts one level
//     lower: rank1(root, row) is never needed because rank1 of every child
//     over the row-indexed image equals its rank over the root's positions.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <string>
#include <functional>
#include <vector>

#include "../../include/mbrwt.h"

namespace mbrwt {

enum : uint8_t {
    KIND_LEAF = 0,
    KIND_PLANE = 1,
    KIND_MASK8 = 2,
    KIND_MASK16 = 3,
    KIND_MASK32 = 4,
    KIND_MASK64 = 5,
    KIND_FOLDED = 6,  // the BRWT root when folded into the super-root (never visited)
    KIND_PACK = 7,    // node whose children are all MASK8 nodes: children bits + their masks inline
    KIND_PACK2 = 8,   // node whose children are all PACK-shaped: the whole 3-level subtree inline
    KIND_PACKT = 9,   // a root child whose whole subtree (any shape) is packed into per-position records
    KIND_PACKT_IN = 10,  // internal node inside a KIND_PACKT subtree (record only, no image)
};
inline bool is_mask_kind(uint8_t k) { return k >= KIND_MASK8 && k <= KIND_MASK64; }

// KIND_PACK image: one 64-byte block per 16 positions.  Quarter q (16 bytes)
// = {u16 bits of child 2q, u16 bits of child 2q+1, 12 bytes of the mask
// area}; the logical 48-byte mask area (quarters' 12-byte segments in order)
// holds the MASK8 mask of every set (child, position) pair of the block,
// child-major, position-ascending.  A block with more than 48 pairs keeps
// the u64 address of a spill list (same order) in area bytes 0..7.  The
// MASK8 children keep their records (labels, arity) but have no image.
constexpr uint32_t kPackSpan = 16;
constexpr uint32_t kPackBlock = 64;
constexpr uint32_t kPackArea = 48;
// byte offset inside a block of logical mask-area byte o
__host__ __device__ inline uint32_t pack_area_byte(uint32_t o) { return 16 * (o / 12) + 4 + o % 12; }

// KIND_PACK2 image (node u whose children A are all PACK-shaped: each A has
// 1..8 MASK8 children B with consecutive leaf columns): one 64-byte block per
// S positions of u, S = the node's span (1, 2, 4 or 8, kept in
// DevNode::stride and as log2 in the CNode's log2(stride) bits).  Bytes
// 0..S-1 = start[t], the byte offset of position t's record (start[0] = S);
// records back to back.  Record of position j =
//   m2                      u's children bits at j (never 0: u's bit is set),
//   m1(A) per set A         A's children bits at A's position (rank1(A, j) - 1),
//   leaf(A,B) per set A, per set B of m1(A), both in child order
//                           B's leaf mask at B's position,
// i.e. the index bits of the whole subtree below u at j, in the reference's
// pre-order (BRWT.cpp:45-51).  A block whose records exceed 64 - S bytes
// holds start[0] = 0 and, in bytes 8..15, the address of a spill list:
// u16 start[S+1] (relative to the list; start[S] = the end) followed by the
// records.  No record is longer than 64 bytes (the fast kernel stages a
// spilled record in a 64-byte LDS slot): the host builder declines PACK2 for
// a node with a longer record, the generator fails loudly (it needs >= 55 of
// a node's <= 64 grandchildren set at one position).  The A and B
// nodes keep their records (arity, first child, labels) but have no image.
// Sparse subtrees take S = 8 (Kingsford shape: ~4.5 record bytes per
// position), dense ones a smaller span (RefSeq shape: ~23 bytes, S = 2).
constexpr uint32_t kPack2MaxSpan = 8;
constexpr uint32_t kPack2Block = 64;
__host__ __device__ inline uint32_t pack2_inline(uint32_t span) { return kPack2Block - span; }
// KIND_PACKT image (node u, a child of the folded root, whose subtree has
// height <= kPacktMaxDepth and arities <= kPacktMaxArity -- any partitioner's
// shape, e.g. the greedy + relaxed trees of the reference's build scripts):
// the blocks and spill lists of KIND_PACK2 with any span S in 1..8, and the
// record of position j = its label count and the index bits of u's whole
// subtree at j in DFS pre-order:
//   count    the number of leaves set below u at j (<= 255; one byte),
//   mask(v)  the children bits of internal node v at v's position (1 byte for
//            arity <= 8, else 2 bytes little-endian), starting with v = u,
//   then, for every set child of v in child order that is internal, its
//   record part (recursively).
// Leaves below u come out in the reference's pre-order (BRWT.cpp:45-51) --
// ascending pre-order labels (the count lets a reader place an item's labels
// before walking it).  Internal nodes below u are KIND_PACKT_IN:
// records (arity, first child, length) without an image.  A record is at
// most 64 bytes (the builders decline / fail loudly otherwise).
constexpr uint32_t kPacktMaxDepth = 8;
constexpr uint32_t kPacktMaxArity = 16;
__host__ __device__ inline uint32_t packt_mask_bytes(uint32_t arity) { return arity <= 8 ? 1u : 2u; }
// FLAG_CONSEC_LABELS (MASK nodes): child c's label = label + c.
// FLAG_MASK_CHILDREN (PLANE nodes): every child is a KIND_MASK8 node with
// consecutive labels, so the fast kernel resolves the children in the
// parent's visit (their mask reads are independent and issued together).
enum : uint8_t { FLAG_CONSEC_LABELS = 1, FLAG_MASK_CHILDREN = 2 };

struct alignas(32) DevNode {
    uint64_t base;         // device address of the children image (internal nodes)
    uint32_t first_child;  // dnode id of child 0 (internal nodes)
    uint32_t label;        // leaf: global column; MASK with FLAG_CONSEC_LABELS: label of child 0
    uint32_t stride;       // KIND_PLANE: bytes per 32-position block
    uint16_t arity;
    uint8_t kind;
    uint8_t flags;
    uint64_t length;       // positions in the image (= length of every child's index column)
};
static_assert(sizeof(DevNode) == 32, "DevNode must be 32 bytes");

// Compact 16-byte node record read by the group kernel (kept in LDS for the
// first kLdsNodes dnodes -- in BFS numbering the internal nodes come first):
//   w0 = base[0:48) | kind[48:51) | flag[51] | log2(stride)[52:56) | arity[56:64)
// flag = FLAG_MASK_CHILDREN for KIND_PLANE, FLAG_CONSEC_LABELS for MASK kinds;
// KIND_PACK2 is stored as kind KIND_PACK with flag 1 (kind bits 48..51 = 0xF).
// For KIND_PACK log2(stride) is 6, for KIND_PACK2 it is log2(span).
struct alignas(16) CNode {
    uint64_t w0;
    uint32_t first_child;
    uint32_t label;
};
static_assert(sizeof(CNode) == 16, "CNode must be 16 bytes");
constexpr uint32_t kLdsNodes = 512;
// P2W table (k_traverse_p2w): u32 words
//   [0] R = arity of dnode 0, [1] nA, [2] nB, [3] 0,
//   R x {base lo, base hi, log2(span), index of the node's first child A},
//   nA x {index (into the B part) of A's first child B},
//   nB x {label of B's child 0}      (B: KIND_MASK8, consecutive labels)
constexpr uint32_t kP2wMaxWords = 1024;
// PTW table (k_traverse_ptw: every child of the folded root a leaf or a
// KIND_PACKT node): u32 words
//   [0] R = arity of dnode 0, [1] nI, [2] nE, [3] max subtree height,
//   R x {base lo, base hi, span, entry}   (entry: bit 31 = leaf, then
//        its global column in bits 0..30; else the PACKT node's local index)
//   nI x {first entry [0:16) | arity [24:29)}   (the internal nodes of the
//        PACKT subtrees, local indices)
//   nE u16 child entries (bit 15 = leaf, global column in bits 0..14; else the child's local index)
constexpr uint32_t kPtwMaxWords = 8192;
constexpr uint32_t kFastMaxDepth = 4;  // PLANE levels the specialised kernel's stack holds

inline CNode compact(const DevNode &d) {
    uint32_t lg = 0;
    while (d.stride && (1u << lg) < d.stride) ++lg;
    CNode c;
    const uint64_t flag = d.kind == KIND_PLANE   ? ((d.flags & FLAG_MASK_CHILDREN) ? 1 : 0)
                          : d.kind == KIND_PACK2 ? 1
                          : d.kind == KIND_PACK  ? 0
                                                 : (d.flags & FLAG_CONSEC_LABELS);
    const uint64_t kind = d.kind == KIND_PACK2 ? KIND_PACK : d.kind;
    c.w0 = (d.base & ((1ull << 48) - 1)) | ((kind & 7) << 48) | (flag << 51) |
           ((uint64_t)(lg & 15) << 52) | ((uint64_t)(d.arity & 0xFF) << 56);
    c.first_child = d.first_child;
    c.label = d.label;
    return c;
}

constexpr uint32_t kMaxArity = 64;       // child masks are held in <= 64 bits
constexpr uint32_t kImagePad = 64;       // bytes of zero padding after every image
constexpr uint64_t kMaxRows = 0xFFFFFFFFull;  // positions are 32-bit in the kernels
constexpr uint64_t kShardRowsMax = 1ull << 31;  // rows per row shard of a larger context (shards.hip)

inline uint32_t plane_stride(uint32_t arity) {  // >= 16: blocks are read as 16-byte pairs
    uint32_t s = 16;
    while (s < 8u * arity) s <<= 1;
    return s;
}
inline uint8_t mask_kind(uint32_t arity) {
    return arity <= 8 ? KIND_MASK8 : arity <= 16 ? KIND_MASK16 : arity <= 32 ? KIND_MASK32 : KIND_MASK64;
}
inline uint32_t mask_bytes(uint8_t kind) { return 1u << (kind - KIND_MASK8); }

// Host-side mirror of the device node table plus ownership of the images.
struct Tree {
    std::vector<DevNode> nodes;             // dnode table (host copy)
    std::vector<void *> images;             // device allocations, one per internal dnode
    std::vector<uint8_t> col_path;          // [num_columns][max_depth] child index path per column
    std::vector<uint32_t> col_leaf;         // dnode of the leaf holding each column
    uint32_t path_len = 0;                  // max_depth stride of col_path
    uint32_t stack_depth = 0;               // max KIND_PLANE dnodes on a root path (incl. super)
    bool folded = false;                    // root folded into the super-root
    bool fast_shape = false;                // eligible for k_traverse_fast (finalize_tree)
    bool lds_complete = false;              // every non-leaf dnode id < kLdsNodes (k_traverse_fast2)
    bool has_pack2 = false;                 // some node is KIND_PACK2
    bool has_mask_children = false;         // some PLANE node has FLAG_MASK_CHILDREN
    uint32_t push_frames = 0;               // max stack frames of the fast kernels (non-TERM PLANE nodes on a path)
    uint32_t lds_records = 0;               // last non-leaf dnode id + 1 (node records worth staging in LDS)
    // k_traverse_p2w (the super-root's children all KIND_PACK2): the compact
    // table it stages in LDS (layout: query.hip "P2W table"), empty otherwise
    std::vector<uint32_t> p2w_table;
    bool has_packt = false;                 // some node is KIND_PACKT (general kernels: lane kernel only)
    std::vector<uint32_t> ptw_table;        // k_traverse_ptw's table (layout above), empty otherwise
    // Leaves are labelled by their PRE-ORDER index (the reference's output
    // order, BRWT.cpp:45-51), so the leaves below any node are consecutive
    // labels whatever the partitioner (greedy trees included); label_perm maps
    // a pre-order index back to the global column (empty = identity, e.g. the
    // basic partitioner).  Kernels emit pre-order indices; the CSR writers map.
    std::vector<uint32_t> label_perm;
    uint32_t max_arity = 0;
    uint64_t num_rows = 0, num_columns = 0, num_relations = 0, num_nodes = 0;
    uint64_t image_bytes = 0;
};

struct Workspace {
    void *buf = nullptr;
    size_t bytes = 0;
};

// ROW RECORDS (rows.hip, DESIGN.md §4 "Row records"): the BRWT's index bits
// regrouped by row.  Every bit of node u's index column at position j belongs
// to exactly one row (the row whose descent reaches u at j, BRWT.cpp:30,43),
// so the bits of a row's whole descent -- the children mask of every internal
// node the row reaches, in DFS pre-order (BRWT.cpp:45-51) -- form the row's
// RECORD, and the records of all rows hold exactly the index bits of the tree.
// get_row(r) is then ONE block read and a walk of the record; the rank1
// remaps of the reference are resolved when the image is built.
//   block (B = 64 or 128 bytes, S rows [b S, b S + S)):
//     bytes 0..S-1  e[t] = offset of row t's entry (< B) | 0x80 if spilled
//     inline entry  [u8 label count < 255][masks: 1 byte for arity <= 8, 2 bytes LE for <= 16]
//     spilled entry [u8 min(count, 255)][u32 LE spill offset in 16-byte units]
//   spill entry (16-byte aligned): [u32 count][u32 mask bytes][masks]
// An empty row (no label) is the one-byte entry [0].
// RWT table (the one-lane walks' tree, read from global memory): u32 words
//   [0] nI internal nodes, [1] nE entries, [2] height (internal levels), [3] 0,
//   nI x {first entry [0:24) | arity [24:32)}      (local index 0 = the BRWT root;
//        r06: 24-bit first entries -- 2^16 columns need more than 2^16 entries)
//   nE u32 entries: bit 31 = leaf + global column in bits 0..30, else the local index
constexpr uint32_t kRowsMaxArity = 64;  // (r06: 16 before; masks of up to 8 bytes)
constexpr uint32_t kRowsMaxHeight = 16;
constexpr uint32_t kRowsOdoLevels = 8;  // internal levels the tree odometer walks (rows.hip rows_walk_tree)
constexpr uint32_t kRowsMaxTableWords = 8192;
enum : int { LAYOUT_AUTO = 0, LAYOUT_NODES = 1, LAYOUT_ROWS = 2, LAYOUT_BOTH = 3 };
struct RowsImage {
    bool ready = false;
    uint32_t B = 64, S = 1;         // block bytes, rows per block
    uint64_t magic = 0;             // row / S = umulhi(row, magic) (S > 1)
    uint64_t num_blocks = 0;
    uint8_t *blocks = nullptr;      // num_blocks * B
    uint8_t *spill = nullptr;       // spill entries (+ B bytes of padding)
    uint64_t spill_cap = 0;         // bytes allocated
    unsigned long long *d_spill_used = nullptr;  // 16-byte units taken (build)
    std::vector<uint32_t> table;    // RWT table (the simple kernels, the direct pass)
    uint32_t *d_table = nullptr;
    uint32_t height = 0;
    std::vector<uint32_t> table2;   // RWT2 table (k_traverse_rows: one word per child, leaf parents inline)
    uint32_t *d_table2 = nullptr;
    uint32_t frames = 0;            // its stack levels
    bool mask1 = false;             // every internal node (leaf parents too) has arity <= 8: one-byte masks
    bool nib = false;               // masks as nibble codes (rows_record.hpp RecMasks; MBRWT_BUILD_ROWS_CODE)
    uint32_t max_arity = 0;         // the widest internal node (masks of (arity + 7) / 8 bytes; r06: up to 64)
    // terminal records (MBRWT_BUILD_ROWS_CODE = 2, r06; rows_record.hpp
    // term_walk): the TT table (host, device) the traversal and the one-lane
    // walks read instead of RWT2 / RWT
    bool term = false;
    std::vector<uint32_t> table3;
    uint32_t *d_table3 = nullptr;
    std::vector<uint32_t> slot_dnode;  // RWT2 entry -> dnode (entry nE: the root)
    std::vector<uint32_t> term_dnode;  // terminal id -> dnode (export)
    // the V accounting of terminal records (rows_count_work): per terminal
    // its chain of ancestor dnodes from the root and their arities
    // (WT: [D, nT, 0, 0], nT x D ids, nT x D arities, nT lengths, nT own arities)
    std::vector<uint32_t> table4;
    uint32_t *d_table4 = nullptr;
    uint32_t uni = 0;               // K internal levels above leaf parents on every path (rows_walk_uni), else 0
    uint64_t bytes = 0;             // blocks + spill used
    uint32_t occ_cap = 0;           // workgroups per CU of k_traverse_rows (0 = the default; MBRWT_BUILD_ROWS_WGS_PER_CU)
    // VARIABLE-LENGTH records (rows_var.hip; dense rows): contiguous records
    // [unit bitmap][unit masks] addressed by 64-byte directory lines of 13 rows
    bool var = false;
    uint32_t var_W = 0;                 // bitmap words (units / 32, rounded up)
    uint32_t var_ustride = 0;           // unit u's first column = u * var_ustride for every unit (0: use the table)
    uint32_t var_G = 0;                 // lanes per row of k_var_decode (0 = from the statistics; MBRWT_BUILD_VAR_LANES)
    std::vector<uint32_t> var_units;    // per unit (leaf parent, DFS order): first column | arity << 16
    std::vector<uint16_t> var_unit_of;  // per dnode: its unit, or 0xFFFF
    std::vector<uint32_t> var_anc;      // per unit: its ancestors' dnodes at levels 0..K-1
    uint8_t *var_lines = nullptr;       // num_rows / 13 lines x 64 bytes
    std::vector<void *> var_chunks;     // the records, one allocation per range of rows
    uint32_t *d_var_units = nullptr, *d_var_anc = nullptr;
    uint16_t *d_unit_of = nullptr;
    uint64_t var_rec_bytes = 0;
    // RECORD CLASSES (rows_class.hip; block layout only): the blocks hold one
    // record per distinct record (S = 1) and classes[] maps row r to its
    // record, class_bits bits per row packed LSB-first in u32 words
    uint32_t *classes = nullptr;
    uint32_t class_bits = 0;
    uint64_t num_classes = 0, class_index_bytes = 0, class_sample_distinct = 0;
    // build statistics
    uint64_t spilled_rows = 0, long_rows = 0, record_bytes = 0, spill_bytes = 0;
};
// the RWT table of a finished node tree; false (and an empty table) when the
// shape is outside the row-record kernels' limits
bool build_rwt_table(const Tree &tree, std::vector<uint32_t> &table, uint32_t &height, uint32_t &max_arity);
bool build_rwt2_table(const Tree &tree, std::vector<uint32_t> &table2, uint32_t &frames,
                      std::vector<uint32_t> *slot_dnode = nullptr);
uint32_t rwt2_uniform_levels(const std::vector<uint32_t> &table2);
// the thread's build layout (mbrwt_set_build_option; AUTO when unset)
int build_layout();
void set_build_layout(int layout);
int thread_build_layout();  // the value set for the calling thread (AUTO when unset)
void set_rows_footprint(int v);  // MBRWT_BUILD_ROWS_FOOTPRINT of the calling thread
int rows_footprint();

// Cross-stream ordering of a context's workspaces.  A *_device call returns
// with work still queued on the caller's stream that reads the context's
// workspaces (compaction, classify pass 1, ...); a later call on ANOTHER
// stream must not overwrite them before that work has run.  Every entry point
// that enqueues work holds a WsFence (under the context mutex): it makes the
// call's stream wait for the previous call's last enqueued work, and records
// the new call's end on leaving (include/mbrwt.h "Threading").
struct WsFenceState {
    hipEvent_t ev = nullptr;
    bool live = false;
};
class WsFence {
  public:
    WsFence(WsFenceState &st, hipStream_t s) : st_(st), s_(s) {
        // a stale error of an earlier, unrelated HIP call in this thread
        // would otherwise be reported by the first launch check of this call
        (void)hipGetLastError();
        if (st_.live && st_.ev) (void)hipStreamWaitEvent(s_, st_.ev, 0);
    }
    ~WsFence() {
        if (st_.ev && hipEventRecord(st_.ev, s_) == hipSuccess) st_.live = true;
    }
    WsFence(const WsFence &) = delete;
    WsFence &operator=(const WsFence &) = delete;

  private:
    WsFenceState &st_;
    hipStream_t s_;
};
inline hipError_t create_fence(WsFenceState &st) {  // on the context's device
    return hipEventCreateWithFlags(&st.ev, hipEventDisableTiming);
}
inline void destroy_fence(WsFenceState &st) {
    if (st.ev) (void)hipEventDestroy(st.ev);
    st.ev = nullptr;
    st.live = false;
}

struct HostPipe;  // hostpipe.cpp: the chunked host-buffer get_rows
void free_host_pipe(HostPipe *p);

struct Ctx {
    int device = 0;
    Tree tree;
    DevNode *d_nodes = nullptr;
    CNode *d_cnodes = nullptr;
    uint32_t *d_p2w = nullptr;          // Tree::p2w_table on the device
    uint32_t *d_ptw = nullptr;          // Tree::ptw_table on the device
    uint32_t *d_label_map = nullptr;    // Tree::label_perm on the device (null = identity)
    uint8_t *d_col_path = nullptr;
    uint32_t *d_col_leaf = nullptr;
    hipStream_t stream = nullptr;       // stream of the host-buffer API
    std::mutex mu;
    WsFenceState fence;                 // orders workspace use across callers' streams

    // reusable device workspace (grown on demand, never inside a timed call
    // once warmed up)
    Workspace ws_temp, ws_counts, ws_ovf, ws_scan, ws_rows, ws_out, ws_sort;
    Workspace ws_cls_off, ws_cls_cols;  // get_labels batch: the rows' CSR
    Workspace ws_class;                 // record classes: the batch's classes (rows_class.hip)
    uint64_t *h_scalars = nullptr;      // pinned: [0] total, [1] overflow count, [2] error
    uint64_t *d_scalars = nullptr;      // device twin
    HostPipe *pipe = nullptr;           // streams, slots and staging of mbrwt_get_rows (lazily created)

    // options
    bool timing = false;
    uint32_t slot_labels = 0;           // 0 = auto
    int kernel_variant = 0;             // MBRWT_OPT_KERNEL (0 = default = 5)
    int rows_walk = 0;                  // MBRWT_OPT_ROWS_WALK (6: the non-odometer walk on uniform trees)
    int64_t test_fail_chunk = -1;       // MBRWT_OPT_TEST_FAIL_CHUNK (test hook: host_get_rows fails at that chunk)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // MBRWT_OPT_COMPACT_CUS (r06, VERDICT r05 #1a): k_compact_tiles on a
    // stream masked to compact_cus of every 32 CUs, ordered after the
    // traversal and before the caller's stream by two events
    uint32_t compact_cus = 0;
    hipStream_t s_compact = nullptr;
    hipEvent_t ev_trav = nullptr, ev_comp = nullptr;
    double timing_ms = 0;
    uint64_t timing_launches = 0;
    int grid_cache = 0;
    // launch geometry of the last rowblock kernel (query.hip): the occupancy
    // query and the LDS attribute are host calls paid once, not per batch
    const void *rb_fn = nullptr;
    size_t rb_lds = 0;
    uint32_t rb_threads = 0;
    int rb_cap = 0;
    int rb_blocks = 0;  // resident workgroups on the device

    // Row shards (rows >= 2^32; DESIGN.md §4 "Rows >= 2^32"): a BRWT restricted
    // to a row range is again a BRWT, so a context over more rows than one
    // image's u32 positions holds sub-contexts over consecutive ranges of
    // shard_rows rows; this context's tree then holds only the totals, and
    // every query routes its rows to the shards (shards.hip)
    std::vector<Ctx *> shards;
    uint64_t shard_rows = 0;
    Workspace ws_sh_keys, ws_sh_local, ws_sh_cnt, ws_sh_sort, ws_sh_tmp;

    // Row records (rows.hip): with `rows.ready` every row query runs on them;
    // `nodes_freed` = the per-node images were dropped after the records were
    // built (layout ROWS), so only the row-record kernels can answer
    RowsImage rows;
    bool nodes_freed = false;
    bool rows_sc_dirty = true;   // the row-record kernels' counters (in ws_counts) need clearing
    std::vector<std::pair<hipEvent_t, hipEvent_t>> async_ev;  // timing of asynchronous calls
    size_t async_used = 0;
    uint64_t rows_sc_at = 0;     // their byte offset in ws_counts

    // mbrwt_ctx_clone: a clone shares image_owner's device image (tree
    // images, tables, row records) and owns only its query state; the owner
    // counts its live clones and, destroyed while any is alive, is freed
    // with the last one (both under the clone mutex, capi.cpp)
    Ctx *image_owner = nullptr;
    int clones = 0;
    bool released = false;
};

// row-record image construction (rows.hip): records of the rows [row0, row0 +
// range.num_rows) written from the node image of `range` (a context over
// those rows, tables uploaded); the first range measured decides the block
// size and rows per block (S must divide `align`: every later range starts at
// a multiple of it).  finish_rows uploads the table and marks the image ready.
struct RowsBuild;
RowsBuild *rows_build_begin(Ctx &top, uint64_t num_rows, uint64_t align, bool auto_layout = false);
int rows_build_range(RowsBuild *rb, Ctx &range, uint64_t row0);
int rows_build_finish(RowsBuild *rb);  // frees rb
uint64_t rows_build_pending_bytes(const RowsBuild *rb, uint64_t rows);
void rows_build_abort(RowsBuild *rb);
void free_rows(RowsImage &r);
// row-record queries (rows.hip)
// d_status != null: asynchronous (no host synchronisation; the call's
// {labels needed, status, sticky status bits} land in d_status on the stream)
int rows_get_rows(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets, uint32_t *d_cols, uint64_t cap,
                  uint64_t *needed, hipStream_t s, uint64_t *d_status = nullptr);
// {need, rc, sticky |= 1 << rc} into a caller's status block on the stream
int rows_set_status(uint64_t *d_status, uint64_t need, int rc, hipStream_t s);
int rows_get_batch(Ctx &c, const uint64_t *d_rows, const uint64_t *d_cols, uint64_t n, uint8_t *d_out, hipStream_t s);
int rows_count_labels(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_counts, hipStream_t s);
int rows_count_work(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *visits, uint64_t *labels, hipStream_t s);
int rows_get_column(Ctx &c, uint64_t column, uint64_t *d_rows, uint64_t rows_cap, uint64_t *rows_needed,
                    hipStream_t s);
// record classes (rows_class.hip): build them over a finished block image of
// n rows (mode -1 auto, 0 never, 1 whenever exact and room), map a batch's
// rows to their classes (into ws_class), get_column over the classes
int rows_classes_build(RowsImage &im, uint64_t n, int mode, uint64_t *sample_distinct, hipStream_t s);
int rows_class_map(Ctx &c, const uint64_t *d_rows, uint64_t n, const uint64_t **mapped, hipStream_t s);
int rows_class_get_column(Ctx &c, uint64_t column, uint64_t *d_rows, uint64_t rows_cap, uint64_t *rows_needed,
                          hipStream_t s);
// variable-length records (rows_var.hip)
struct VarScratch {
    Workspace units, cnt, off, acc, scan;
};
bool var_prepare(const Tree &tree, RowsImage &im);  // the unit tables; false when the tree is not uniform
int var_measure_range(RowsImage &im, const Ctx &range, VarScratch &ws, uint64_t *rec_bytes, hipStream_t s);
// the decode's LDS holds a mean tile of such rows beside the tree's unit table
bool var_lds_fits(const RowsImage &im, double labels_per_row, double record_bytes_per_row);
int var_build_range(RowsImage &im, const Ctx &range, uint64_t row0, VarScratch &ws, hipStream_t s);
void var_free_scratch(VarScratch &ws);
int var_get_rows(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets, uint32_t *d_cols, uint64_t cap,
                 uint64_t *needed, hipStream_t s, uint64_t *d_status);
int var_get_batch(Ctx &c, const uint64_t *d_rows, const uint64_t *d_cols, uint64_t n, uint8_t *d_out, hipStream_t s);
// count_labels (d_counts != null) or the V / L accounting (d_counts == null)
int var_count(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_counts, uint64_t *visits, uint64_t *labels,
              hipStream_t s);
int var_get_column(Ctx &c, uint64_t column, uint64_t *d_rows, uint64_t rows_cap, uint64_t *rows_needed,
                   hipStream_t s);

// status helpers ---------------------------------------------------------
void set_error(const std::string &msg);
int hip_fail(hipError_t e, const char *what);

#define MBRWT_HIP(call)                                          \
    do {                                                         \
        hipError_t _e = (call);                                  \
        if (_e != hipSuccess) return ::mbrwt::hip_fail(_e, #call); \
    } while (0)

int ensure(Workspace &w, size_t bytes);

// image construction (image.cpp / synth.hip)
int build_from_desc(const mbrwt_tree_desc &desc, int device, Tree &tree);
// a row shard of a synthetic tree: rows [row0, row0 + desc.num_rows) of the
// whole tree, node u's positions starting at pos0[u] (empty = 0); len_out
// (may be null) receives every internal node's positions in the shard
struct SynthShard {
    uint64_t row0 = 0;
    std::vector<uint64_t> pos0;
    std::vector<uint64_t> *len_out = nullptr;
};
int build_synthetic(const mbrwt_synth_desc &desc, const mbrwt_shape_desc *shape, int device, Tree &tree,
                    hipStream_t stream, const SynthShard *shard = nullptr);
// row shards (shards.hip): rows per shard for a context over num_rows rows
// (0 = one image); MBRWT_SHARD_ROWS forces smaller shards (tests)
uint64_t shard_rows_for(uint64_t num_rows);
// the description of rows [a, b) of a tree (every node's index column cut to
// the positions of those rows); MBRWT_ERR_INVALID when the columns' sizes do
// not nest
struct SlicedDesc {
    std::vector<uint64_t> sizes;
    std::vector<std::vector<uint64_t>> words;
    std::vector<const uint64_t *> ptrs;
    mbrwt_tree_desc desc{};
};
int slice_desc(const mbrwt_tree_desc &in, uint64_t a, uint64_t b, SlicedDesc &out);
int sharded_get_rows(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets, uint32_t *d_cols, uint64_t cap,
                     uint64_t *needed, hipStream_t s);
int sharded_get_batch(Ctx &c, const uint64_t *d_rows, const uint64_t *d_cols, uint64_t n, uint8_t *d_out,
                      hipStream_t s);
int sharded_count_labels(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_counts, hipStream_t s);
int sharded_count_work(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *visits, uint64_t *labels, hipStream_t s);
int sharded_get_column(Ctx &c, uint64_t column, uint64_t *d_rows, uint64_t rows_cap, uint64_t *rows_needed,
                       hipStream_t s);
// the device builders' output: a tree description handed to a sink (the
// image builder, or -- rows >= 2^32 -- the row-sharded / ranged create)
using DescSink = std::function<int(const mbrwt_tree_desc &)>;
int desc_from_columns(const mbrwt_columns_desc &desc, int device, hipStream_t stream, uint64_t relax_max_arity,
                      const DescSink &emit);
int relaxed_desc(const mbrwt_tree_desc &desc, uint64_t max_arity, int device, hipStream_t stream,
                 const DescSink &emit);
// the calling thread's partitioner for build_from_columns (mbrwt_set_build_option)
int build_partitioner();
void set_build_partitioner(int partitioner);
int build_from_columns(const mbrwt_columns_desc &desc, int device, Tree &tree, hipStream_t stream,
                       uint64_t relax_max_arity = 0);
// BRWTOptimizer::relax on a tree description (build.hip)
int build_relaxed_from_desc(const mbrwt_tree_desc &desc, uint64_t max_arity, int device, Tree &tree,
                            hipStream_t stream);
void free_tree(Tree &tree);
// finish a Tree whose nodes/images are set: column paths, stack depth
int finalize_tree(Tree &tree);
// the P2W table of k_traverse_p2w (empty when the tree has another shape)
void build_p2w_table(Tree &tree);
// the PTW table of k_traverse_ptw (empty when the tree has another shape)
void build_ptw_table(Tree &tree);

// the calling thread's tuning / test build options (include/mbrwt.h
// MBRWT_BUILD_ROWS_VAR .. MBRWT_BUILD_ROWS_CLASSES; every default automatic)
struct BuildTuning {
    int rows_var = -1;           // -1 auto, 0 never, 1 always
    uint32_t var_lanes = 0;      // 0 auto
    uint32_t rows_block = 0;     // 0 auto, else B << 8 | S
    uint64_t rows_range = 0;     // 0 auto
    uint32_t node_kinds = 15;    // MBRWT_KIND_* bits
    uint64_t shard_rows = 0;     // 0: the default shard size
    uint32_t rows_wgs_per_cu = 0;
    int rows_classes = -1;       // record classes: -1 auto, 0 never, 1 whenever exact
    int rows_code = 0;           // records: 0 AUTO (terminal records where smaller, else byte masks), 1 nibble codes, 2 terminal records, 3 byte masks
};
BuildTuning &build_tuning();
void set_build_tuning(const BuildTuning &t);

inline bool fold_root_enabled() { return (build_tuning().node_kinds & 1u) != 0; }
inline bool pack_enabled() { return (build_tuning().node_kinds & 2u) != 0; }
inline bool pack2_enabled() { return pack_enabled() && (build_tuning().node_kinds & 4u) != 0; }
inline bool packt_enabled() { return pack_enabled() && (build_tuning().node_kinds & 8u) != 0; }

// queries (query.hip)
// column query (column.hip): ascending rows of `column` into d_rows (u64)
int run_get_column(Ctx &c, uint64_t column, uint64_t *d_rows, uint64_t rows_cap, uint64_t *rows_needed,
                   hipStream_t s);
const char *traverse_kernel_name(const Ctx &c);  // the kernel mbrwt_get_rows* launches
// mbrwt_get_rows: host row ids -> host CSR, chunked and pipelined (hostpipe.cpp)
int host_get_rows(Ctx &c, const uint64_t *rows, uint64_t n, uint64_t *offsets, uint32_t *cols, uint64_t cols_cap,
                  uint64_t *cols_needed);
int run_get_rows(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets, uint32_t *d_cols, uint64_t cap,
                 uint64_t *needed, hipStream_t s);
int run_get_batch(Ctx &c, const uint64_t *d_rows, const uint64_t *d_cols, uint64_t n, uint8_t *d_out, hipStream_t s);
int run_count_labels(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *d_counts, hipStream_t s);
// batched get_labels(indices, presence_ratio) (classify.hip)
// the classify driver, shared by both schemes (classify.hip): the rows'
// labels come from `get_rows` (device CSR; MBRWT_ERR_CAPACITY + need when
// cols_cap is too small), workspaces from the scheme's context
struct ClassifyIo {
    Workspace *off, *cols, *cnt, *scan;
};
using ClassifyRowsFn = std::function<int(uint64_t *d_off, uint32_t *d_cols, uint64_t cols_cap, uint64_t *need)>;
int classify_labels(const ClassifyIo &io, const ClassifyRowsFn &get_rows, uint64_t m, uint64_t n_rows,
                    const uint64_t *d_read_off, uint64_t n_reads, double ratio, uint64_t *d_lab_off, uint32_t *d_labels,
                    uint64_t cap, uint64_t *needed, hipStream_t s);
int classify_top_labels(const ClassifyIo &io, const ClassifyRowsFn &get_rows, uint64_t m, uint64_t n_rows,
                        const uint64_t *d_read_off, uint64_t n_reads, uint64_t num_top, uint64_t *d_lab_off,
                        uint32_t *d_labels, uint64_t *d_counts, uint64_t cap, uint64_t *needed, hipStream_t s);
int run_get_labels_batch(Ctx &c, const uint64_t *d_rows, uint64_t n_rows, const uint64_t *d_read_off, uint64_t n_reads,
                         double ratio, uint64_t *d_lab_off, uint32_t *d_labels, uint64_t cap, uint64_t *needed,
                         hipStream_t s);
int run_get_top_labels_batch(Ctx &c, const uint64_t *d_rows, uint64_t n_rows, const uint64_t *d_read_off,
                             uint64_t n_reads, uint64_t num_top, uint64_t *d_lab_off, uint32_t *d_labels,
                             uint64_t *d_counts, uint64_t cap, uint64_t *needed, hipStream_t s);
int run_count_work(Ctx &c, const uint64_t *d_rows, uint64_t n, uint64_t *visits, uint64_t *labels, hipStream_t s);

}  // namespace mbrwt

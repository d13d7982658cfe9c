/*
 * mbrwt.h -- C ABI of the MI355X-native Multi-BRWT row-query engine
 * (genome_graph_annotation_amd/libmbrwt.so).
 *
 * Drop-in boundary for the reference's BRWT query path
 * (ratschlab/genome_graph_annotation; paths below are relative to its root):
 *
 *   reference                                        replaced by
 *   -----------------------------------------------  -----------------------------------
 *   BinaryMatrix::get_row        common/binary_matrix.hpp:21      mbrwt_get_rows / _device (batched)
 *   BRWT::get_row                annotation/hierarchical_annotation/BRWT.cpp:26-53
 *   BRWT::get                    BRWT.cpp:9-24                     mbrwt_get_batch / _device
 *   BRWT::get_column             BRWT.cpp:55-85 (select1,          mbrwt_get_column / _device
 *                                bit_vector.cpp:863-869)
 *   bit_vector_rrr<63>::rank1    common/bit_vector.cpp:857-861     (inside the traversal kernel)
 *   bit_vector_rrr<63>::operator[]  common/bit_vector.cpp:884-888  (inside the traversal kernel)
 *   utils::RangePartition::get   common/utils.cpp:689-691          (leaf column table, composed)
 *   BRWT::num_rows/num_columns   BRWT.hpp:33-34                    mbrwt_num_rows / mbrwt_num_columns
 *   BRWT::num_relations          BRWT.cpp:130-140                  mbrwt_num_relations
 *   BRWT::load (structure ingestion) BRWT.cpp:87-111               mbrwt_create (from a tree description)
 *   StaticBinRelAnnotator::count_labels annotation/annotate_static.cpp:149-162
 *                                                                  mbrwt_count_labels_device
 *
 * Conventions: plain pointers and sizes only; no C++ or torch types.  Every
 * function returns an MBRWT_* status code; nothing throws across the ABI.
 * Rows are uint64 (binary_matrix.hpp:11) and must be < mbrwt_num_rows().
 * Columns are emitted as uint32 (the reference stores them as uint32,
 * utils.hpp:442-444).  Output order per row is the reference's order: the
 * pre-order (DFS) of the BRWT's leaves (BRWT.cpp:45-51).
 *
 * Threading: a context may be used from several host threads; calls on one
 * context are serialised internally (the reference's get_row is const and
 * called concurrently from a ThreadPool, main.cpp:462-497).  Device-buffer
 * calls (*_device) may return with work still queued on the caller's stream;
 * the context orders its internal workspaces across streams (each call's
 * stream waits for the previous call's queued work, whichever stream that was
 * on), so calls on different streams are safe.  The caller's own output
 * buffers are ready when the caller's stream reaches them.
 */
#ifndef MBRWT_H
#define MBRWT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define MBRWT_OK 0
#define MBRWT_ERR_INVALID 1     /* bad argument or malformed tree description */
#define MBRWT_ERR_RANGE 2       /* row or column out of range (reference: assert, BRWT.cpp:27) */
#define MBRWT_ERR_CAPACITY 3    /* cols_cap too small; *cols_needed holds the size needed */
#define MBRWT_ERR_UNSUPPORTED 4 /* tree beyond this build's limits */
#define MBRWT_ERR_DEVICE 5      /* HIP runtime error (see mbrwt_last_error_message) */
#define MBRWT_ERR_NOMEM 6       /* device or host allocation failed */

typedef struct mbrwt_ctx mbrwt_ctx;

/* ---- structure ingestion ---------------------------------------------- */
/*
 * A BRWT in breadth-first numbering: node 0 is the root; the children of node
 * u are nodes [first_child[u], first_child[u] + num_children[u]) in the
 * reference's child order (BRWT.hpp:60).  vec_words[u] points to node u's
 * index column (BRWT.hpp:59 nonzero_rows_) as ceil(vec_size[u]/64) LSB-first
 * uint64 words.  For a leaf, leaf_column[u] is the global column id obtained by
 * composing RangePartition::get along the path (utils.cpp:689-691); internal
 * nodes carry UINT32_MAX.  num_nodes == 0 describes the empty BRWT().
 * Replaces BRWT::load (BRWT.cpp:87-111) as the way structure enters the engine.
 */
typedef struct mbrwt_tree_desc {
    uint64_t num_rows;
    uint64_t num_columns;
    uint32_t num_nodes;
    const uint32_t *num_children;
    const uint32_t *first_child;
    const uint32_t *leaf_column;
    const uint64_t *vec_size;
    const uint64_t *const *vec_words;
} mbrwt_tree_desc;

/* Build the device image of a BRWT on HIP device `device`. */
int mbrwt_create(const mbrwt_tree_desc *desc, int device, mbrwt_ctx **out);

/*
 * Generate a synthetic Multi-BRWT directly in device memory: the law of a
 * basic-partitioner (BRWT_builders.cpp:20-31) BRWT built from i.i.d.
 * Bernoulli(density) columns (experiments/data_generation.cpp:20-29), drawn
 * top-down from a counter-based hash (spec: DESIGN.md "Synthetic matrices").
 * arity in [2, 12]; num_rows >= 2^32 builds row shards (mbrwt_num_shards).
 */
typedef struct mbrwt_synth_desc {
    uint64_t num_rows;
    uint64_t num_columns;
    double density;
    uint32_t arity;
    uint64_t seed;
} mbrwt_synth_desc;
int mbrwt_create_synthetic(const mbrwt_synth_desc *desc, int device, mbrwt_ctx **out);

/*
 * The same law over ANY tree shape (e.g. the shape of a greedy + relaxed tree,
 * the reference's production build path: transform_anno --greedy then
 * relax_brwt): BFS arrays as in mbrwt_tree_desc (children contiguous,
 * leaf_column = the leaf's global column, UINT32_MAX for internal nodes),
 * node arity <= 12; desc->arity is ignored and desc->num_columns must equal
 * the number of leaves.  q(u) = 1 - (1-density)^(leaves below u); node keys
 * are BFS ids.
 */
typedef struct mbrwt_shape_desc {
    uint32_t num_nodes;
    const uint32_t *num_children;
    const uint32_t *first_child;
    const uint32_t *leaf_column;
} mbrwt_shape_desc;
int mbrwt_create_synthetic_shaped(const mbrwt_synth_desc *desc, const mbrwt_shape_desc *shape, int device,
                                  mbrwt_ctx **out);

/*
 * Build a BRWT from its columns on the device: BRWTBottomUpBuilder::build
 * (BRWT_builders.cpp:119-163) with the basic partitioner of the given arity
 * (get_basic_partitioner, BRWT_builders.cpp:20-31; groups of one pass
 * through).  compute_or and generate_subindex run as HIP kernels; the result
 * is the image mbrwt_create would build from the same tree.  columns[j] is
 * column j over the rows as ceil(num_rows/64) LSB-first uint64 words in host
 * memory (bits past num_rows are ignored).  arity in [2, 64]; num_columns == 0
 * gives the empty BRWT().
 */
typedef struct mbrwt_columns_desc {
    uint64_t num_rows;
    uint64_t num_columns;
    const uint64_t *const *columns;
    uint32_t arity;
} mbrwt_columns_desc;
int mbrwt_create_from_columns(const mbrwt_columns_desc *desc, int device, mbrwt_ctx **out);

/*
 * BRWTOptimizer::relax(brwt, max_arity) (BRWT_builders.cpp:166-297;
 * `annograph relax_brwt --relax-arity`, main.cpp:746, config.cpp:104):
 * internal nodes whose removal saves space (pruning_delta, :351-380, with the
 * RRR size model of :315-321) are removed and their children re-attached to
 * the parent, within max_arity children per node.  The re-attached children's
 * index columns are expanded on the device.  Query results are unchanged.
 * mbrwt_create_from_columns_relaxed = mbrwt_create_from_columns then relax
 * (the reference's convert + relax_brwt); mbrwt_create_relaxed relaxes an
 * exported tree.  max_arity <= 1 leaves the tree as built.
 */
int mbrwt_create_from_columns_relaxed(const mbrwt_columns_desc *desc, uint64_t relax_max_arity, int device,
                                      mbrwt_ctx **out);
int mbrwt_create_relaxed(const mbrwt_tree_desc *desc, uint64_t max_arity, int device, mbrwt_ctx **out);

void mbrwt_destroy(mbrwt_ctx *ctx);

/* A second query context over the SAME device image (no copy): its own
 * workspaces, status block, events and host-buffer stream, so queries on a
 * context and on its clones may run concurrently on different streams (or
 * host threads) -- the reference's server answers concurrent requests from
 * one annotator (cli/server.cpp); calls on ONE context are ordered on its
 * workspace fence.  Options start at their defaults.  Destroying the source
 * while clones are alive defers the image's release to the last clone.
 * Sharded contexts clone their shards.  Replaces nothing in the reference:
 * its annotator is shared by reference across its worker threads. */
int mbrwt_ctx_clone(mbrwt_ctx *src, mbrwt_ctx **out);

/* ---- device layout ------------------------------------------------------
 * Two layouts of the same tree:
 *   NODES  per-node, sibling-interleaved index columns with ranks; get_row is
 *          the reference's rank1 descent (BRWT.cpp:26-53) over them;
 *   ROWS   ROW RECORDS: the tree's index bits regrouped by row (each row's
 *          descent -- the children mask of every internal node it reaches, in
 *          DFS pre-order -- stored with the row), so get_row is one block read
 *          and a record walk; the rank1 remaps are resolved at build time.
 *          Trees with arity <= 64 (r06; 16 before: nodes wider than 16
 *          need a tree of at most 8 internal levels), < 2^16 columns (2^15
 *          before), height <= 16.  Built one
 *          range of rows at a time, so rows >= 2^32 need no row shards.
 *          get_column scans the records; mbrwt_tree_export rebuilds every
 *          index column from the records (so BinaryMatrix::serialize works).
 *   BOTH   both images: get_rows / count_labels on the records, the rest on
 *          the node image.
 * The layout is chosen when a context is created: mbrwt_set_build_option
 * (MBRWT_BUILD_LAYOUT, value) sets it for the mbrwt_create* / mbrwt_load calls
 * of the calling thread; MBRWT_LAYOUT_AUTO (the default) chooses: ROWS when
 * the tree is within the row-record limits, its records cost at most ~1.25
 * block requests per row (no dense-row shapes) and the image fits the
 * device, NODES otherwise.  Layout ROWS on a tree outside its limits ->
 * MBRWT_ERR_UNSUPPORTED.  No reference counterpart (the reference's BRWT has
 * one sdsl layout).
 */
#define MBRWT_BUILD_LAYOUT 1
/* (MBRWT_BUILD_PARTITIONER, value): the partitioner of the calling thread's
   mbrwt_create_from_columns[_relaxed] -- MBRWT_PARTITIONER_BASIC (default:
   groups of desc->arity consecutive nodes) or MBRWT_PARTITIONER_GREEDY
   (binary_grouping_greedy, partitionings.cpp:148-196, the `--greedy` build of
   scripts/kingsford/convert.sh:24; desc->arity is ignored): per level the
   inner products of every column pair over the reference's row sample
   (min(10^6, rows) rows, mt19937 seed 1) on the device, the candidate sort
   and the matching on the host as the reference does them. */
#define MBRWT_BUILD_PARTITIONER 2
#define MBRWT_PARTITIONER_BASIC 0
#define MBRWT_PARTITIONER_GREEDY 1
/* (MBRWT_BUILD_ROWS_FOOTPRINT, value): how the calling thread's row-record
   builds pick the block size and rows per block -- MBRWT_ROWS_FAST (default:
   the fewest modelled requests per row, then the smallest image within 2 %)
   or MBRWT_ROWS_COMPACT (the smallest image within 30 % of the fewest
   modelled requests: the greedy + relax shape at 3.7 B rows takes 158.90 GB
   instead of 236.85 GB for a 2 % slower kernel). */
#define MBRWT_BUILD_ROWS_FOOTPRINT 3
#define MBRWT_ROWS_FAST 0
#define MBRWT_ROWS_COMPACT 1
#define MBRWT_LAYOUT_AUTO 0
#define MBRWT_LAYOUT_NODES 1
#define MBRWT_LAYOUT_ROWS 2
#define MBRWT_LAYOUT_BOTH 3
/* Tuning and test options of the calling thread's builds (r05: these were
   environment variables read by the library; they are now explicit, scoped
   like the options above).  Every default is the automatic choice.
   MBRWT_BUILD_ROWS_VAR       -1 auto, 0 never, 1 always the variable-length
                              records of dense rows (uniform trees)
   MBRWT_BUILD_VAR_LANES      lanes per row of their decode (0 auto; 1..16, a
                              power of two)
   MBRWT_BUILD_ROWS_BLOCK     row-record blocks: 0 auto, else B << 8 | S (B 64 or
                              128 bytes, S rows per block)
   MBRWT_BUILD_ROWS_RANGE     rows per range of a ranged row-record build (0
                              auto; a multiple of 360,360)
   MBRWT_BUILD_NODE_KINDS     node-image kinds built (bit mask, default all):
                              MBRWT_KIND_FOLD_ROOT | _PACK | _PACK2 | _PACKT;
                              PACK2 / PACKT also need PACK
   MBRWT_BUILD_SHARD_ROWS     rows per row shard (0: 2^31; small values force
                              shards on small trees -- a test hook)
   MBRWT_BUILD_ROWS_WGS_PER_CU  resident workgroups per CU of the row-record
                              traversal (0 auto; occupancy sweeps)
   MBRWT_BUILD_ROWS_CLASSES   RECORD CLASSES of the block layout:
                              one copy of every distinct row record plus a
                              class index of ceil(log2 classes) bits per row,
                              for data whose rows repeat few label sets.
                              -1 auto (default: built when a tenth of a
                              2^20-row sample repeats a record, kept when
                              there are at most half as many classes as rows
                              and they at least halve the image), 0 never,
                              1 whenever they fit (always exact: every row's
                              record is compared with its class's)
   MBRWT_BUILD_ROWS_CODE      how a row record stores the row's descent
                              (DESIGN §4g, §4h): 0 (default) AUTO -- TERMINAL
                              RECORDS where they are smaller than byte masks,
                              else byte masks; 1 NIBBLE CODES -- a mask with
                              one bit set as that bit's index in 4 bits, any
                              other as 12 bits -- for uniform trees of arity
                              <= 8 (other trees keep bytes); 2 terminal
                              records where they fit: the leaf parents and
                              leaves the descent reaches, in pre-order, each
                              a field {id, its children mask} (masks <= 16
                              bits, <= 4,096 terminals); 3 one byte per 8
                              children of every internal node reached */
#define MBRWT_BUILD_ROWS_VAR 4
#define MBRWT_BUILD_VAR_LANES 5
#define MBRWT_BUILD_ROWS_BLOCK 6
#define MBRWT_BUILD_ROWS_RANGE 7
#define MBRWT_BUILD_NODE_KINDS 8
#define MBRWT_BUILD_SHARD_ROWS 9
#define MBRWT_BUILD_ROWS_WGS_PER_CU 10
#define MBRWT_BUILD_ROWS_CLASSES 11
#define MBRWT_BUILD_ROWS_CODE 12
#define MBRWT_KIND_FOLD_ROOT 1
#define MBRWT_KIND_PACK 2
#define MBRWT_KIND_PACK2 4
#define MBRWT_KIND_PACKT 8
#define MBRWT_KIND_ALL 15
int mbrwt_set_build_option(int option, int64_t value);
/* The calling thread's current value of a build option (so that a caller can
   restore it after a scoped change). */
int mbrwt_get_build_option(int option, int64_t *value);
int mbrwt_layout(const mbrwt_ctx *ctx); /* MBRWT_LAYOUT_NODES / _ROWS / _BOTH of a context */
/* Row-record image: out[0] block bytes B (0: the variable-length records of
   dense rows -- then [1] = 13 rows per directory line, [2] directory bytes),
   [1] rows per block S, [2] block
   bytes, [3] spill bytes, [4] record bytes (counts + masks), [5] spilled rows,
   [6] rows longer than a block, [7] tree height | K << 32, K = the internal
   levels above the leaf parents when every path has that many (the
   odometer walk of csrc/rows.hip), else 0.  MBRWT_ERR_UNSUPPORTED without
   row records. */
int mbrwt_rows_stats(const mbrwt_ctx *ctx, uint64_t out[8]);
/* Record classes of a row-record image: out[0] classes (0: none -- then the
   blocks hold one record per row), [1] class index bits per row, [2] class
   index bytes, [3] distinct records in the layout-AUTO sample (0: not
   sampled).  With classes, mbrwt_rows_stats describes the dictionary (one
   record per class, S = 1).  MBRWT_ERR_UNSUPPORTED without row records. */
int mbrwt_rows_classes(const mbrwt_ctx *ctx, uint64_t out[4]);

/* ---- multi-device (one process, N GPUs) --------------------------------
 * A replica of the tree on every device of `devices` (n entries; a device
 * may repeat), built concurrently with the calling thread's build layout,
 * and get_rows over a batch cut into n contiguous slices -- slice r on
 * replica r -- reassembled into the caller's ONE CSR: host buffers
 * (mbrwt_multi_get_rows: device-to-host copies at each slice's label offset)
 * or device buffers on devices[0] (mbrwt_multi_get_rows_device: peer copies
 * over xGMI, `stream` on devices[0]).  Results, order and the capacity
 * protocol are those of mbrwt_get_rows over the whole batch.  The
 * reference's `annograph classify` runs its ThreadPool in one process
 * (main.cpp:462-497): this is how its host drives every GPU of a node.
 * mbrwt_multi_replica gives replica i's context (point / column queries,
 * properties, export); it is owned by the multi handle.
 */
typedef struct mbrwt_multi mbrwt_multi;
int mbrwt_multi_create(const mbrwt_tree_desc *desc, const int *devices, int n, mbrwt_multi **out);
int mbrwt_multi_create_synthetic(const mbrwt_synth_desc *desc, const int *devices, int n, mbrwt_multi **out);
int mbrwt_multi_load(const uint8_t *bytes, uint64_t len, uint64_t *consumed, const int *devices, int n,
                     mbrwt_multi **out);
void mbrwt_multi_destroy(mbrwt_multi *m);
int mbrwt_multi_size(const mbrwt_multi *m);
mbrwt_ctx *mbrwt_multi_replica(mbrwt_multi *m, int i);
int mbrwt_multi_get_rows(mbrwt_multi *m, const uint64_t *rows, uint64_t n, uint64_t *offsets, uint32_t *cols,
                         uint64_t cols_cap, uint64_t *cols_needed);
int mbrwt_multi_get_rows_device(mbrwt_multi *m, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets,
                                uint32_t *d_cols, uint64_t cols_cap, uint64_t *cols_needed, void *stream);

/* ---- files: the reference's BRWT stream (the matrix of a .brwt.annodbg) ----
 * An owned tree description (host memory).  Byte formats of sdsl-lite /
 * libmaus2 are restated from their published algorithms: PARITY UNPINNED
 * (no sdsl source or reference-written file exists here).
 *
 * mbrwt_tree_parse      BRWT::load (BRWT.cpp:87-111): the pre-order stream of
 *                       {RangePartition (utils.cpp:702-715), rrr_vector<63>
 *                       index (bit_vector.cpp:906-925), child count, children}
 *                       starting at bytes[0]; *consumed (may be NULL) = bytes
 *                       read.  MBRWT_ERR_INVALID on a malformed stream (the
 *                       reference's load returns false).  Host only, no GPU.
 * mbrwt_tree_serialize  BRWT::serialize (BRWT.cpp:113-128) of a description:
 *                       capacity protocol as mbrwt_get_rows (buf may be NULL
 *                       for the sizing call).  Host only, no GPU.
 * mbrwt_tree_export     the tree a context holds, read back from its device
 *                       image (every node's index column; any image layout).
 * mbrwt_load            mbrwt_tree_parse + mbrwt_create.
 */
typedef struct mbrwt_tree mbrwt_tree;
int mbrwt_tree_parse(const uint8_t *bytes, uint64_t len, uint64_t *consumed, mbrwt_tree **out);
int mbrwt_tree_serialize(const mbrwt_tree_desc *desc, uint8_t *buf, uint64_t cap, uint64_t *needed);
int mbrwt_tree_export(mbrwt_ctx *ctx, mbrwt_tree **out);
const mbrwt_tree_desc *mbrwt_tree_get_desc(const mbrwt_tree *tree); /* valid until mbrwt_tree_free */
void mbrwt_tree_free(mbrwt_tree *tree);
int mbrwt_load(const uint8_t *bytes, uint64_t len, uint64_t *consumed, int device, mbrwt_ctx **out);

/* ---- properties (BRWT.hpp:33-51) -------------------------------------- */
uint64_t mbrwt_num_rows(const mbrwt_ctx *ctx);
uint64_t mbrwt_num_columns(const mbrwt_ctx *ctx);
uint64_t mbrwt_num_relations(const mbrwt_ctx *ctx);
uint64_t mbrwt_num_nodes(const mbrwt_ctx *ctx);
uint64_t mbrwt_device_bytes(const mbrwt_ctx *ctx); /* HBM held by the structure image */
int mbrwt_device(const mbrwt_ctx *ctx);
/*
 * Row shards: the reference's Row is uint64_t (binary_matrix.hpp:11).  One
 * device image addresses < 2^32 positions, so a context over more rows
 * (mbrwt_create, mbrwt_load, mbrwt_create_synthetic[_shaped]) holds row
 * shards of 2^31 rows -- each the BRWT restricted to its row range -- and
 * routes every query's rows to them; results are those of the whole matrix.
 * mbrwt_num_shards = 1 for an ordinary context.  (The build option
 * MBRWT_BUILD_SHARD_ROWS forces smaller shards: a test hook.)
 */
uint64_t mbrwt_num_shards(const mbrwt_ctx *ctx);

/* ---- queries ----------------------------------------------------------- */
/*
 * Batched BRWT::get_row over rows[0..n): CSR result with offsets[0..n]
 * (n+1 entries, offsets[0] = 0) and cols[offsets[i]..offsets[i+1]) = row i's
 * column ids in the reference's order.  If the total exceeds cols_cap,
 * returns MBRWT_ERR_CAPACITY with *cols_needed set to the total (retry
 * protocol); offsets and cols are then unspecified (a prefix of the CSR
 * may have been written).  cols_needed may be NULL.  Host buffers: the
 * batch is cut into chunks of 2^20 rows whose upload, query and download
 * overlap (r05, hostpipe.cpp); page-locked buffers (hipHostMalloc,
 * hipHostRegister) are read and written by DMA directly, pageable ones are
 * staged through the context's pinned buffers by a pool of host threads.
 */
int mbrwt_get_rows(mbrwt_ctx *ctx, const uint64_t *rows, uint64_t n, uint64_t *offsets, uint32_t *cols,
                   uint64_t cols_cap, uint64_t *cols_needed);

/*
 * Same on device buffers (d_rows: n uint64; d_offsets: n+1 uint64; d_cols:
 * cols_cap uint32), enqueued on HIP stream `stream` (hipStream_t, NULL =
 * default stream).  The call synchronises `stream` once to learn the output
 * size; the results are complete when `stream` is next synchronised.
 */
int mbrwt_get_rows_device(mbrwt_ctx *ctx, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets,
                          uint32_t *d_cols, uint64_t cols_cap, uint64_t *cols_needed, void *stream);

/*
 * The same without any host synchronisation, for pipelines that keep the
 * device busy (consecutive batches, the multi-GPU exchange): the call only
 * enqueues work on `stream`.  When the stream reaches its end, d_status
 * (device memory, 3 uint64) holds {labels needed, MBRWT_* status of the
 * call, sticky bits |= 1 << status} -- the caller clears word 2 and checks
 * it after synchronising.  Over cols_cap the status is MBRWT_ERR_CAPACITY
 * and no label is written past cols_cap (offsets may be); out-of-range rows give
 * MBRWT_ERR_RANGE.  The return value reports only argument and launch errors.
 * On a per-node image the call runs the synchronous path (one host sync)
 * and then writes the same status block.
 */
int mbrwt_get_rows_device_async(mbrwt_ctx *ctx, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets,
                                uint32_t *d_cols, uint64_t cols_cap, uint64_t *d_status, void *stream);

/* Batched BRWT::get (BRWT.cpp:9-24): out[i] = bit (rows[i], cols[i]). Host buffers. */
int mbrwt_get_batch(mbrwt_ctx *ctx, const uint64_t *rows, const uint64_t *cols, uint64_t n, uint8_t *out);
int mbrwt_get_batch_device(mbrwt_ctx *ctx, const uint64_t *d_rows, const uint64_t *d_cols, uint64_t n,
                           uint8_t *d_out, void *stream);

/*
 * BRWT::get_column (BRWT.cpp:55-85; BinaryMatrix::get_column,
 * binary_matrix.hpp:21): the ascending rows carrying `column`, written to
 * rows[0..*rows_needed).  If the column has more than rows_cap rows, returns
 * MBRWT_ERR_CAPACITY with *rows_needed set and rows untouched (call with
 * rows_cap = 0 to size the buffer).  column >= num_columns -> MBRWT_ERR_RANGE
 * (an assert in the reference).  Host buffer / device buffer + stream.
 */
int mbrwt_get_column(mbrwt_ctx *ctx, uint64_t column, uint64_t *rows, uint64_t rows_cap, uint64_t *rows_needed);
int mbrwt_get_column_device(mbrwt_ctx *ctx, uint64_t column, uint64_t *d_rows, uint64_t rows_cap,
                            uint64_t *rows_needed, void *stream);

/*
 * StaticBinRelAnnotator::count_labels (annotate_static.cpp:149-162) fused on
 * the device: counts[c] (num_columns uint64, zeroed by the call) = number of
 * rows among d_rows[0..n) that carry column c.  Device buffers.
 */
int mbrwt_count_labels_device(mbrwt_ctx *ctx, const uint64_t *d_rows, uint64_t n, uint64_t *d_counts,
                              void *stream);

/*
 * StaticBinRelAnnotator::get_labels(indices, presence_ratio)
 * (annotate_static.cpp:71-94) for many reads at once -- the `classify`
 * consumer of get_rows.  Read r's row indices are
 * d_rows[d_read_offsets[r] .. d_read_offsets[r+1]) (n_reads + 1 ascending
 * offsets, the first 0, the last n_rows); its labels are the columns present
 * in at least ceil(len_r * presence_ratio) of its rows (in >= 1 row when the
 * ratio is 0), ascending.  Output: d_label_offsets[n_reads + 1] and d_labels
 * (capacity protocol as mbrwt_get_rows: MBRWT_ERR_CAPACITY + labels_needed).
 * presence_ratio outside [0, 1] (an assert in the reference) ->
 * MBRWT_ERR_INVALID; more than 15,360 columns -> MBRWT_ERR_UNSUPPORTED.
 * Device buffers + stream; mbrwt_get_labels_batch is the host-buffer form
 * (read_offsets validated as on the device: ascending, last = n_rows).
 */
int mbrwt_get_labels_batch(mbrwt_ctx *ctx, const uint64_t *rows, uint64_t n_rows, const uint64_t *read_offsets,
                           uint64_t n_reads, double presence_ratio, uint64_t *label_offsets, uint32_t *labels,
                           uint64_t labels_cap, uint64_t *labels_needed);
int mbrwt_get_labels_batch_device(mbrwt_ctx *ctx, const uint64_t *d_rows, uint64_t n_rows,
                                  const uint64_t *d_read_offsets, uint64_t n_reads, double presence_ratio,
                                  uint64_t *d_label_offsets, uint32_t *d_labels, uint64_t labels_cap,
                                  uint64_t *labels_needed, void *stream);

/*
 * MultiLabelEncoded::get_top_labels(indices, num_top) (annotate.cpp:57-83;
 * `classify --count-labels`, main.cpp:177) for many reads at once: read r's
 * labels present in >= 1 of its rows with their row counts, by count
 * descending, at most num_top of them.  Equal counts come in ascending label
 * order (the reference's std::sort leaves their order unspecified).  Reads as
 * mbrwt_get_labels_batch; output d_label_offsets[n_reads + 1], d_labels (u32)
 * and d_counts (u64) side by side, labels_cap entries each (capacity protocol
 * as mbrwt_get_rows).  More than 8,192 columns -> MBRWT_ERR_UNSUPPORTED.
 */
int mbrwt_get_top_labels_batch(mbrwt_ctx *ctx, const uint64_t *rows, uint64_t n_rows, const uint64_t *read_offsets,
                               uint64_t n_reads, uint64_t num_top, uint64_t *label_offsets, uint32_t *labels,
                               uint64_t *counts, uint64_t labels_cap, uint64_t *labels_needed);
int mbrwt_get_top_labels_batch_device(mbrwt_ctx *ctx, const uint64_t *d_rows, uint64_t n_rows,
                                      const uint64_t *d_read_offsets, uint64_t n_reads, uint64_t num_top,
                                      uint64_t *d_label_offsets, uint32_t *d_labels, uint64_t *d_counts,
                                      uint64_t labels_cap, uint64_t *labels_needed, void *stream);

/* ---- measurement ------------------------------------------------------- */
/*
 * Roofline accounting (DESIGN.md "Measurement"): over rows[0..n) (device
 * buffer) return sum V(row) (index-bit probes the reference recursion makes,
 * BRWT.cpp:30) and sum L(row) (labels returned).  Untimed diagnostic pass.
 */
int mbrwt_count_work_device(mbrwt_ctx *ctx, const uint64_t *d_rows, uint64_t n, uint64_t *sum_visits,
                            uint64_t *sum_labels, void *stream);

/* Options (mbrwt_set_option). */
/* ---- multi-GPU exchange helpers --------------------------------------- */
/*
 * Bit-packing of n values < 2^bits (bits in 1..32) into ceil(n*bits/32) u32
 * words (value i at bits [i*bits, (i+1)*bits), LSB-first), and back; device
 * buffers, launched on `stream`.  The all-gatherv that reassembles a sharded
 * batch's CSR (genome_graph_annotation_amd/dist.py) ships labels and row
 * counts at ceil(log2(num_columns)) bits with these.  No reference
 * counterpart (the reference has no multi-GPU path).
 */
int mbrwt_pack_ids_device(const uint32_t *d_values, uint64_t n, uint32_t bits, uint32_t *d_words, void *stream);
int mbrwt_unpack_ids_device(const uint32_t *d_words, uint64_t n, uint32_t bits, uint32_t *d_values, void *stream);
/* The unpacking of a whole all-gathered wire buffer in one launch: segment r
   (r < nseg) starts at d_base + r * seg_stride bytes (a multiple of 4) and
   holds counts[r] (host array) packed values; they are written to d_values
   back to back in segment order. */
int mbrwt_unpack_segments_device(const void *d_base, uint32_t nseg, uint64_t seg_stride, const uint64_t *counts,
                                 uint32_t bits, uint32_t *d_values, void *stream);
/* The all-gatherv with DEVICE-side sizes (no host synchronisation per
   exchange; dist.py AllGatherV(device_sizes=True)).  A rank's wire segment of
   `wire_bytes` (a multiple of 16) is
     [u64 num_labels][n_rows row counts at bits_count][zero pad to 16 bytes]
     [min(num_labels, labels_cap) labels at bits_label][zero pad]
   with both fields in whole chunks of 32 values (a chunk = bits words;
   value i at bits [i*bits, (i+1)*bits) of the field, LSB-first)
   with num_labels read from the device (*d_num_labels, e.g. word 0 of the
   status block of mbrwt_get_rows_device_async) and the row counts taken
   from the CSR offsets (offsets[i+1] - offsets[i]); d_cols holds cols_cap
   labels: num_labels > cols_cap (the rank's get_rows failed on capacity, its
   CSR unwritten) writes the header 2^64 - 1 and nothing else, so the unpack
   flags the exchange; the label field starts
   at byte labels_offset (a multiple of 16, at least
   mbrwt_wire_labels_offset(n_rows, bits_count): every rank of an exchange
   uses the offset of the largest slice) and needs
   ceil(labels_cap / 32) * bits_label words.
   MBRWT_ERR_INVALID when the layout does not fit wire_bytes. */
uint64_t mbrwt_wire_labels_offset(uint64_t n_rows, uint32_t bits_count);
int mbrwt_pack_csr_device(const uint64_t *d_offsets, uint64_t n_rows, const uint32_t *d_cols, uint64_t cols_cap,
                          const uint64_t *d_num_labels, uint64_t labels_cap, uint32_t bits_count, uint32_t bits_label,
                          uint64_t labels_offset, void *d_wire, uint64_t wire_bytes, void *stream);
/* The labels of every segment of an all-gathered buffer of such segments
   (segment r at d_base + r * seg_stride; its label field at labels_offset
   bytes), written back to back in segment order: the segments' label counts
   and their prefix are read from the headers ON THE DEVICE.  d_status[0] =
   the total, d_status[1] = 0, or 1 when a header exceeds labels_cap or the
   total exceeds values_cap (nothing is written then). */
int mbrwt_unpack_labels_device(const void *d_base, uint32_t nseg, uint64_t seg_stride, uint64_t labels_offset,
                               uint64_t labels_cap, uint32_t bits, uint32_t *d_values, uint64_t values_cap,
                               uint64_t *d_status, void *stream);

/* The global CSR offsets of an all-gathered wire straight from its packed
   row counts (r04): d_offsets[0 .. N] = the exclusive prefix of every
   segment's counts (segment r: counts[r] values of `bits` bits each at byte
   8 of d_base + r * seg_stride, the layout mbrwt_pack_csr_device writes),
   N = sum(counts) -- block sums, one workgroup's scan of them, then every
   block's counts re-read and scanned in LDS (no int32 count array in
   between).  d_temp == NULL: *temp_bytes receives the
   scratch size the call needs and nothing runs.  At most 8 segments (one
   node); MBRWT_ERR_UNSUPPORTED beyond (unpack the counts and scan them). */
int mbrwt_unpack_offsets_device(const void *d_base, uint32_t nseg, uint64_t seg_stride, const uint64_t *counts,
                                uint32_t bits, uint64_t *d_offsets, void *d_temp, uint64_t *temp_bytes,
                                void *stream);

#define MBRWT_OPT_TIMING 1       /* 1: time the traversal kernel with HIP events */
#define MBRWT_OPT_SLOT_LABELS 2  /* per-row label slots of the fast path (0 = auto) */
#define MBRWT_OPT_KERNEL 4       /* traversal kernel (A/B measurement): 0 default (k_traverse_p2w, else
                                    k_traverse_fast2 where eligible, else the group kernel), 1 lane-per-row,
                                    2/3/4 group with 1/2/4 children per lane, 5/6 group at 8/6 waves per
                                    SIMD, 10 group + non-temporal reads, 17/18 k_traverse_fast2 plain /
                                    non-temporal, 19/20 k_traverse_p2w plain / non-temporal, 24..30
                                    k_traverse_ptw configurations (each falls back to the next kernel where
                                    the tree is not eligible); others rejected.  Node images only. */
#define MBRWT_OPT_ROWS_WALK 8  /* row records: 0 default (the odometer walk over the path table on uniform
                                   trees, the tree odometer on every other shape of <= 8 internal levels),
                                   3 the tree odometer, 4 the stack walk, 6 the stack walk of one-byte masks,
                                   7 the odometer without the path table (A/B and tests) */
#define MBRWT_OPT_COMPACT_CUS 64 /* row records (r06, measurement): 0 default; k in 1..31 runs the
                                    compaction of get_rows_device on a stream masked to k of every 32 CUs
                                    (hipExtStreamCreateWithCUMask), after the traversal and before the
                                    caller's stream by two events */
#define MBRWT_OPT_TEST_FAIL_CHUNK 32 /* test hook: mbrwt_get_rows (host buffers) fails with MBRWT_ERR_NOMEM
                                        when it reaches chunk `value` of the batch (-1: never) -- the error
                                        path's drain of the chunks already in flight is tested with it */
int mbrwt_set_option(mbrwt_ctx *ctx, int option, int64_t value);

/* Traversal-kernel time accumulated while MBRWT_OPT_TIMING is on (ms, launches); resets the sums. */
int mbrwt_take_timing(mbrwt_ctx *ctx, double *kernel_ms, uint64_t *launches);

const char *mbrwt_strerror(int status);
const char *mbrwt_last_error_message(void); /* thread-local detail of the last failure */

/* Diagnostics: name of the traversal kernel mbrwt_get_rows* launches for this
   tree under the current MBRWT_OPT_KERNEL (static string; "" for a null ctx). */
const char *mbrwt_traverse_kernel(mbrwt_ctx *ctx);

#ifdef __cplusplus
}
#endif

#endif /* MBRWT_H */

/*
 * mbrwt_wt.h -- C ABI of the device BinRel-WT engine (SURVEY.md §8(f) row 1:
 * BinRel-WT(sdsl) get_row, BASELINE configs[4]).  Same conventions as
 * mbrwt.h (status codes, capacity protocol, host and device-buffer variants).
 *
 * Reference interface this replaces (ratschlab/genome_graph_annotation):
 *   BinRelWT_sdsl(generate_rows, num_relations,   annotation/bin_rel_wt/bin_rel_wt_sdsl.cpp:10-40
 *                 num_columns)                     -> mbrwt_wt_create (CSR rows instead of a callback)
 *   BinRelWT_sdsl::num_rows/num_columns/           bin_rel_wt_sdsl.cpp:42-49, :161-163
 *                 num_relations                    -> mbrwt_wt_num_*
 *   BinRelWT_sdsl::get_row                         bin_rel_wt_sdsl.cpp:51-83   -> mbrwt_wt_get_rows[_device]
 *   BinRelWT_sdsl::get                             bin_rel_wt_sdsl.cpp:98-109  -> mbrwt_wt_get_batch[_device]
 *   BinRelWT_sdsl::get_column                      bin_rel_wt_sdsl.cpp:85-96   -> mbrwt_wt_get_column[_device]
 *   BinRelWT_sdsl::load / serialize                bin_rel_wt_sdsl.cpp:113-132 -> mbrwt_wt_load / mbrwt_wt_serialize
 *
 * Semantics: rows are sets of column ids (BinaryMatrix rows).  get_row
 * returns the row's ids ascending (sdsl wt_int::interval_symbols order);
 * get_column the rows carrying the id, ascending.  A row listing the same id
 * twice is rejected at creation (MBRWT_ERR_INVALID): the reference asserts
 * nothing there and would return padding zeros / repeated rows.
 */
#ifndef MBRWT_WT_H
#define MBRWT_WT_H

#include "mbrwt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mbrwt_wt mbrwt_wt;

/* CSR rows: row r's column ids are cols[offsets[r] .. offsets[r+1]) in any
 * order; offsets has num_rows + 1 entries, offsets[0] = 0. */
typedef struct mbrwt_binrel_desc {
    uint64_t num_rows;
    uint64_t num_columns;
    const uint64_t *offsets;
    const uint32_t *cols;
} mbrwt_binrel_desc;

/* Synthetic i.i.d. Bernoulli(density) matrix generated on the device
 * (DESIGN.md "BinRel-WT": cell (r, c) set iff mix64(K(r) + c * 0xD1B54A32D192ED03)
 * < density * 2^64, K(r) = mix64(seed ^ ((r + 1) * 0x9E3779B97F4A7C15))). */
typedef struct mbrwt_binrel_synth_desc {
    uint64_t num_rows;
    uint64_t num_columns;
    double density;
    uint64_t seed;
} mbrwt_binrel_synth_desc;

int mbrwt_wt_create(const mbrwt_binrel_desc *desc, int device, mbrwt_wt **out);
int mbrwt_wt_create_synthetic(const mbrwt_binrel_synth_desc *desc, int device, mbrwt_wt **out);
void mbrwt_wt_destroy(mbrwt_wt *ctx);

uint64_t mbrwt_wt_num_rows(const mbrwt_wt *ctx);
uint64_t mbrwt_wt_num_columns(const mbrwt_wt *ctx);
uint64_t mbrwt_wt_num_relations(const mbrwt_wt *ctx);
uint64_t mbrwt_wt_device_bytes(const mbrwt_wt *ctx);

/* Batched get_row -> CSR (offsets[n+1] u64, cols u32); capacity protocol as mbrwt_get_rows. */
int mbrwt_wt_get_rows(mbrwt_wt *ctx, const uint64_t *rows, uint64_t n, uint64_t *offsets, uint32_t *cols,
                      uint64_t cols_cap, uint64_t *cols_needed);
int mbrwt_wt_get_rows_device(mbrwt_wt *ctx, const uint64_t *d_rows, uint64_t n, uint64_t *d_offsets,
                             uint32_t *d_cols, uint64_t cols_cap, uint64_t *cols_needed, void *stream);

/* Batched get: out[i] = bit (rows[i], cols[i]). */
int mbrwt_wt_get_batch(mbrwt_wt *ctx, const uint64_t *rows, const uint64_t *cols, uint64_t n, uint8_t *out);
int mbrwt_wt_get_batch_device(mbrwt_wt *ctx, const uint64_t *d_rows, const uint64_t *d_cols, uint64_t n,
                              uint8_t *d_out, void *stream);

/* get_column: ascending rows carrying `column`; capacity protocol as mbrwt_get_column. */
int mbrwt_wt_get_column(mbrwt_wt *ctx, uint64_t column, uint64_t *rows, uint64_t rows_cap, uint64_t *rows_needed);
int mbrwt_wt_get_column_device(mbrwt_wt *ctx, uint64_t column, uint64_t *d_rows, uint64_t rows_cap,
                               uint64_t *rows_needed, void *stream);

/* MBRWT_OPT_TIMING only: HIP-event time of the decode kernel of get_rows. */
/*
 * Batched classify over a BinRel-WT matrix: get_labels(indices,
 * presence_ratio) (annotate_static.cpp:71-94) and get_top_labels(indices,
 * num_top) (annotate.cpp:57-83) for many reads; arguments, output and errors
 * exactly as mbrwt_get_labels_batch[_device] / mbrwt_get_top_labels_batch[_device]
 * in mbrwt.h (the same device kernels behind mbrwt_wt_get_rows_device).
 */
int mbrwt_wt_get_labels_batch(mbrwt_wt *ctx, const uint64_t *rows, uint64_t n_rows, const uint64_t *read_offsets,
                              uint64_t n_reads, double presence_ratio, uint64_t *label_offsets, uint32_t *labels,
                              uint64_t labels_cap, uint64_t *labels_needed);
int mbrwt_wt_get_labels_batch_device(mbrwt_wt *ctx, const uint64_t *d_rows, uint64_t n_rows,
                                     const uint64_t *d_read_offsets, uint64_t n_reads, double presence_ratio,
                                     uint64_t *d_label_offsets, uint32_t *d_labels, uint64_t labels_cap,
                                     uint64_t *labels_needed, void *stream);
int mbrwt_wt_get_top_labels_batch(mbrwt_wt *ctx, const uint64_t *rows, uint64_t n_rows, const uint64_t *read_offsets,
                                  uint64_t n_reads, uint64_t num_top, uint64_t *label_offsets, uint32_t *labels,
                                  uint64_t *counts, uint64_t labels_cap, uint64_t *labels_needed);
int mbrwt_wt_get_top_labels_batch_device(mbrwt_wt *ctx, const uint64_t *d_rows, uint64_t n_rows,
                                         const uint64_t *d_read_offsets, uint64_t n_reads, uint64_t num_top,
                                         uint64_t *d_label_offsets, uint32_t *d_labels, uint64_t *d_counts,
                                         uint64_t labels_cap, uint64_t *labels_needed, void *stream);

/*
 * The reference's file stream (BinRelWT_sdsl::load / serialize,
 * bin_rel_wt_sdsl.cpp:113-132): {num_columns as a libmaus2 number, the
 * concatenated rows' ids as sdsl wt_int<rrr_vector<63>>, bit_vector_rrr
 * delimiters -- a 1, then per row a 0 per id and a 1}.  Byte layouts restated
 * from sdsl-lite's / libmaus2's published formats: PARITY UNPINNED (DESIGN.md
 * §13).  Host only except mbrwt_wt_load (creates a device context) and
 * mbrwt_wt_serialize (reads a context's rows back, ids ascending per row).
 *
 * mbrwt_wt_parse         stream -> an owned CSR (mbrwt_binrel_get_desc);
 *                        MBRWT_ERR_INVALID on a malformed stream (the
 *                        reference's load returns false); *consumed = bytes read
 * mbrwt_wt_serialize_desc  CSR -> stream, ids in the given order; capacity
 *                        protocol as mbrwt_tree_serialize (buf may be NULL)
 */
typedef struct mbrwt_binrel mbrwt_binrel;
int mbrwt_wt_parse(const uint8_t *bytes, uint64_t len, uint64_t *consumed, mbrwt_binrel **out);
const mbrwt_binrel_desc *mbrwt_binrel_get_desc(const mbrwt_binrel *b);
void mbrwt_binrel_free(mbrwt_binrel *b);
int mbrwt_wt_serialize_desc(const mbrwt_binrel_desc *desc, uint8_t *buf, uint64_t cap, uint64_t *needed);
int mbrwt_wt_load(const uint8_t *bytes, uint64_t len, uint64_t *consumed, int device, mbrwt_wt **out);
int mbrwt_wt_serialize(mbrwt_wt *ctx, uint8_t *buf, uint64_t cap, uint64_t *needed);

int mbrwt_wt_set_option(mbrwt_wt *ctx, int option, int64_t value);
int mbrwt_wt_take_timing(mbrwt_wt *ctx, double *kernel_ms, uint64_t *launches);

#ifdef __cplusplus
}
#endif

#endif /* MBRWT_WT_H */

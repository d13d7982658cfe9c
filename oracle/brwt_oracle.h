/*
 * brwt_oracle.h -- C ABI of the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * The oracle is a CPU restatement of the reference's BRWT / Multi-BRWT query
 * path (ratschlab/genome_graph_annotation).  It exists to check the HIP product
 * path and to time the CPU baseline.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle.so; the product library
 * (genome_graph_annotation_amd/libmbrwt.so) never links or calls it.
 *
 * Each function cites the reference file:line whose behaviour it restates
 * (paths relative to the reference repository root).
 */
#ifndef BRWT_ORACLE_H
#define BRWT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct OracleTree OracleTree;

/* ---- construction ------------------------------------------------------ */

/* BRWTBottomUpBuilder::build (annotation/hierarchical_annotation/BRWT_builders.cpp:122-163)
 * over `num_cols` columns of `num_rows` bits each.  Column j's bits are the
 * LSB-first u64 words col_words[j * ceil(num_rows/64) ...].
 * partitioner: 0 = get_basic_partitioner(arity) (BRWT_builders.cpp:20-31),
 *              1 = binary_grouping_greedy (partitionings.cpp:148-201).
 * relax_max_arity > 1 additionally runs BRWTOptimizer::relax (BRWT_builders.cpp:166-211);
 * pass UINT64_MAX for the unbounded relax of tests/test_BRWT_optimizer.cpp. */
OracleTree *oracle_build_from_columns(const uint64_t *col_words, uint64_t num_rows,
                                      uint64_t num_cols, int partitioner, uint32_t arity,
                                      uint64_t relax_max_arity);

/* `run_experiments matrices simulate norepl` (experiments/main.cpp:216-231):
 * DataGenerator seeded `seed` draws `num_cols` Bernoulli(density) columns
 * column-major from one std::mt19937 (experiments/data_generation.cpp:20-29,
 * :103-110), then builds as oracle_build_from_columns. */
uint64_t oracle_generate_uniform_rows(uint64_t n, uint64_t m, double d, uint64_t unique, uint32_t seed,
                                      uint64_t *col_words);
uint64_t oracle_generate_uniform_columns(uint64_t n, uint64_t m, double d, uint64_t unique, uint32_t seed,
                                         uint64_t *col_words);
uint64_t oracle_rrr_bytes(OracleTree *t);
OracleTree *oracle_generate_norepl(uint64_t num_rows, uint64_t num_cols, double density,
                                   uint32_t seed, int partitioner, uint32_t arity,
                                   uint64_t relax_max_arity);

/* Top-down synthetic Multi-BRWT of the basic-partitioner shape (DESIGN.md
 * "Synthetic matrices"): the law of a BRWT built from i.i.d. Bernoulli(density)
 * columns, drawn node by node from a counter-based hash.  num_threads <= 0 = all. */
OracleTree *oracle_generate_topdown(uint64_t num_rows, uint64_t num_cols, double density,
                                    uint32_t arity, uint64_t seed, int num_threads);

void oracle_free(OracleTree *t);

/* BRWT::get_row (BRWT.cpp:26-53) over the top-down synthetic tree of the same
 * spec WITHOUT materialising it: every index bit is a pure function of (node,
 * position), so each node with queries streams its child masks up to its
 * largest queried position, counting per child for the inclusive rank1
 * (BRWT.cpp:30,43).  Memory O(batch x depth): used for the parity checks of
 * sizes whose plain index bits exceed host RAM (1 B x 3,173 = 158 GB).
 * *status = 0, or 2 on an out-of-range row (then NULL).  The CSR holds each
 * row's columns in the reference's order. */
typedef struct OracleCSR OracleCSR;
OracleCSR *oracle_topdown_get_rows(uint64_t num_rows, uint64_t num_cols, double density,
                                   uint32_t arity, uint64_t seed, const uint64_t *rows,
                                   uint64_t n, int num_threads, int *status);
/* The same two entry points over ANY tree shape (BFS arrays as
 * mbrwt_shape_desc: num_children, first_child, leaf_column): the law of a BRWT
 * of that shape over i.i.d. Bernoulli(density) columns (q(u) = 1 - (1-d)^cols(u)),
 * node keys = BFS ids.  NULL / *status = 1 on a malformed shape. */
OracleCSR *oracle_topdown_get_rows_shaped(uint64_t num_rows, uint32_t num_nodes, const uint32_t *num_children,
                                          const uint32_t *first_child, const uint32_t *leaf_column, double density,
                                          uint64_t seed, const uint64_t *rows, uint64_t n, int num_threads,
                                          int *status);
OracleTree *oracle_generate_topdown_shaped(uint64_t num_rows, uint32_t num_nodes, const uint32_t *num_children,
                                           const uint32_t *first_child, const uint32_t *leaf_column, double density,
                                           uint64_t seed, int num_threads);
uint64_t oracle_csr_num_labels(const OracleCSR *r);
uint64_t oracle_csr_draws(const OracleCSR *r);  /* mask draws streamed */
void oracle_csr_copy(const OracleCSR *r, uint64_t *offsets /* n+1 */, uint32_t *cols);
void oracle_csr_free(OracleCSR *r);

/* ---- BinaryMatrix surface (common/binary_matrix.hpp:9-29, BRWT.hpp:33-51) -- */
uint64_t oracle_num_rows(const OracleTree *t);
uint64_t oracle_num_columns(const OracleTree *t);
uint64_t oracle_num_relations(const OracleTree *t);      /* BRWT.cpp:130-140 */
uint64_t oracle_num_nodes(const OracleTree *t);          /* BRWT.cpp:161-167 */
double oracle_avg_arity(const OracleTree *t);            /* BRWT.cpp:142-159 */
uint64_t oracle_total_column_size(const OracleTree *t);  /* BRWT.cpp:184-192 */
uint64_t oracle_total_num_set_bits(const OracleTree *t); /* BRWT.cpp:194-202 */
uint32_t oracle_depth(const OracleTree *t);

/* BRWT::get (BRWT.cpp:9-24).  Returns 0/1; -1 if out of range. */
int oracle_get(const OracleTree *t, uint64_t row, uint64_t col);

/* BRWT::get_row (BRWT.cpp:26-53): writes up to `cap` column ids in the
 * reference's output order and returns the row's label count (may exceed cap).
 * *visits (optional) receives V(row) = number of index-bit probes
 * (operator[] calls, BRWT.cpp:30) the recursion makes. */
uint64_t oracle_get_row(const OracleTree *t, uint64_t row, uint32_t *out, uint64_t cap,
                        uint64_t *visits);

/* Batched get_row over rows[0..n) -> CSR (offsets[n+1], cols).  Returns 0 on
 * success, 1 if cols_cap is too small (then *cols_needed is set and cols is
 * untouched), 2 on an out-of-range row.  visits/labels (optional, per row)
 * receive V(row) and L(row).  num_threads <= 0 = all (OpenMP dynamic). */
int oracle_get_rows(const OracleTree *t, const uint64_t *rows, uint64_t n,
                    uint64_t *offsets, uint32_t *cols, uint64_t cols_cap,
                    uint64_t *cols_needed, uint32_t *visits, int num_threads);

/* Timing-only batched get_row (the CPU baseline): runs the reference
 * recursion over rows[0..n) on num_threads threads and returns the total
 * label count (results are discarded, as in experiments/main.cpp:78-93). */
uint64_t oracle_time_rows(const OracleTree *t, const uint64_t *rows, uint64_t n,
                          int num_threads);

/* BRWT::get_column (BRWT.cpp:55-85): returns count, writes up to cap rows. */
uint64_t oracle_get_column(const OracleTree *t, uint64_t col, uint64_t *out, uint64_t cap);

/* The CPU baseline's sdsl-RRR-like leg: re-encode every node's index as
 * 63-bit blocks {class, combinatorial number} with rank / pointer samples
 * every 32 blocks (the cost model of bit_vector_rrr<63>,
 * bit_vector.cpp:857-888) and drop the plain bits.  Afterwards only
 * oracle_get / oracle_get_row(s) / oracle_time_rows are valid. */
void oracle_to_rrr(OracleTree *t, int num_threads);

/* ---- export in BFS numbering (the layout of include/mbrwt.h's tree desc) -- */
uint32_t oracle_export_num_nodes(const OracleTree *t);
/* arrays of length oracle_export_num_nodes(); leaf_column = UINT32_MAX for
 * internal nodes; children of node u are [first_child[u], first_child[u]+num_children[u]). */
void oracle_export(const OracleTree *t, uint32_t *num_children, uint32_t *first_child,
                   uint32_t *leaf_column, uint64_t *vec_size);
/* Pointer to node u's index-vector words (LSB-first, ceil(size/64) words). */
const uint64_t *oracle_export_vec_words(const OracleTree *t, uint32_t node);

/* ---- data generation (experiments/data_generation.cpp) ----------------- */
/* generate_random_ints (data_generation.cpp:7-18) with DataGenerator seeded
 * `seed`; note the reference's std::uniform_int_distribution<> is `int`. */
void oracle_generate_random_ints(uint64_t n, uint64_t begin, uint64_t end, uint32_t seed,
                                 uint64_t *out);
/* Column-major Bernoulli matrix exactly as generate_random_columns draws it
 * (data_generation.cpp:20-29, :103-110); output packed like col_words above. */
void oracle_generate_columns(uint64_t num_rows, uint64_t num_cols, double density,
                             uint32_t seed, uint64_t *col_words);

/* ---- bit-vector primitives (common/bit_vector.hpp:12-45) for KATs ------- */
typedef struct OracleBitVec OracleBitVec;
OracleBitVec *oracle_bv_new(const uint64_t *words, uint64_t size);
void oracle_bv_free(OracleBitVec *bv);
uint64_t oracle_bv_rank1(const OracleBitVec *bv, uint64_t id);   /* bit_vector.cpp:857-861 */
uint64_t oracle_bv_select1(const OracleBitVec *bv, uint64_t i);  /* bit_vector.cpp:863-869 */
int oracle_bv_get(const OracleBitVec *bv, uint64_t id);          /* bit_vector.cpp:884-888 */
uint64_t oracle_bv_num_set_bits(const OracleBitVec *bv);

/* ---- synthetic-spec helpers (shared spec with the product) ---- */
uint64_t oracle_synth_hash(uint64_t seed, uint64_t key, uint64_t pos);

#ifdef __cplusplus
}
#endif

#endif /* BRWT_ORACLE_H */

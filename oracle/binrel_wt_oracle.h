/*
 * binrel_wt_oracle.h -- C ABI of the BinRel-WT(sdsl) CPU oracle
 * (TEST INFRASTRUCTURE ONLY; same rules as brwt_oracle.h: only tests/,
 * __graft_entry__.smoke() and the CPU-baseline legs may load it).
 *
 * Restates annotation/bin_rel_wt/bin_rel_wt_sdsl.{hpp,cpp} (reference) over
 * a levelwise wavelet tree with the published semantics of
 * sdsl::wt_int<rrr_vector<63>> (hmusta/sdsl-lite fork, commit not recorded in
 * the reference snapshot; .gitmodules:18-21): rank(i, c) counts c in [0, i),
 * select(k, c) is the position of the k-th c (1-based), interval_symbols(i, j)
 * lists the distinct symbols of [i, j) in ascending order.
 */
#ifndef BINREL_WT_ORACLE_H
#define BINREL_WT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct OracleWT OracleWT;

/* BinRelWT_sdsl(generate_rows, num_relations, num_columns)
 * (bin_rel_wt_sdsl.cpp:10-40) over CSR rows: row r's column ids are
 * cols[offsets[r] .. offsets[r+1]) in the order generate_rows would emit them.
 * Returns NULL if a column id is >= num_columns (an assert in the reference). */
OracleWT *wt_oracle_build(const uint64_t *offsets, const uint32_t *cols, uint64_t num_rows, uint64_t num_columns);
/* the empty constructor (bin_rel_wt_sdsl.hpp:11): delimiters_(1, 1) */
OracleWT *wt_oracle_empty(void);
void wt_oracle_free(OracleWT *t);

uint64_t wt_oracle_num_rows(const OracleWT *t);       /* bin_rel_wt_sdsl.cpp:46-49 */
uint64_t wt_oracle_num_columns(const OracleWT *t);    /* :42-44 */
uint64_t wt_oracle_num_relations(const OracleWT *t);  /* :161-163 */

/* get_row (bin_rel_wt_sdsl.cpp:51-83): writes the (last - first) entries the
 * reference returns (distinct symbols ascending, then zeros if the row had
 * repeated ids) up to cap; returns the entry count, UINT64_MAX if out of range. */
uint64_t wt_oracle_get_row(const OracleWT *t, uint64_t row, uint32_t *out, uint64_t cap);
/* get (bin_rel_wt_sdsl.cpp:98-109): 0/1, -1 if out of range. */
int wt_oracle_get(const OracleWT *t, uint64_t row, uint64_t col);
/* get_column (bin_rel_wt_sdsl.cpp:85-96): rows in occurrence order; returns
 * the count (may exceed cap), UINT64_MAX if out of range. */
uint64_t wt_oracle_get_column(const OracleWT *t, uint64_t col, uint64_t *out, uint64_t cap);

/* Batched get_row -> CSR (offsets[n+1], cols); 0 ok, 1 capacity (cols_needed
 * set), 2 out of range.  num_threads <= 0 = all. */
int wt_oracle_get_rows(const OracleWT *t, const uint64_t *rows, uint64_t n, uint64_t *offsets, uint32_t *cols,
                       uint64_t cols_cap, uint64_t *cols_needed, int num_threads);
/* wall seconds of get_row over rows[0..n) on num_threads (CPU baseline) */
double wt_oracle_time_rows(const OracleWT *t, const uint64_t *rows, uint64_t n, int num_threads);

/* Synthetic i.i.d. Bernoulli(density) row (DESIGN.md "BinRel-WT"): the set
 * columns of row `row`, ascending; cell (r, c) is set iff
 * mix64(K(r) + c * 0xD1B54A32D192ED03) < threshold, K(r) = mix64(seed ^
 * ((r + 1) * 0x9E3779B97F4A7C15)), threshold = wt_synth_threshold(density).
 * Writes up to cap ids and returns the row's count. */
uint64_t wt_synth_threshold(double density);
uint64_t wt_synth_row(uint64_t row, uint64_t num_columns, uint64_t threshold, uint64_t seed, uint32_t *out,
                      uint64_t cap);
/* CSR of synthetic rows [row0, row0 + n): offsets[n+1] (relative), cols. */
int wt_synth_rows(uint64_t row0, uint64_t n, uint64_t num_columns, double density, uint64_t seed, uint64_t *offsets,
                  uint32_t *cols, uint64_t cols_cap, uint64_t *cols_needed, int num_threads);
/* Same for arbitrary rows[0..n) (any order, repeats allowed): the rows of the
 * full-size parity checks, row-independent by construction. */
int wt_synth_rows_at(const uint64_t *rows, uint64_t n, uint64_t num_columns, double density, uint64_t seed,
                     uint64_t *offsets, uint32_t *cols, uint64_t cols_cap, uint64_t *cols_needed,
                     int num_threads);

#ifdef __cplusplus
}
#endif

#endif

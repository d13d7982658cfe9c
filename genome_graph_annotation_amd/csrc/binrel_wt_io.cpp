// binrel_wt_io.cpp -- BinRelWT_sdsl::load / serialize (annotation/bin_rel_wt/
// bin_rel_wt_sdsl.cpp:113-132) for the device BinRel-WT engine: the stream is
// {libmaus2 number num_columns, sdsl wt_int<rrr_vector<63>> of the
// concatenated rows' column ids, bit_vector_rrr delimiters (a 1, then per row
// one 0 per id and a 1: the ctor, bin_rel_wt_sdsl.cpp:10-40)}.  Parsing and
// writing are host-only; mbrwt_wt_load / mbrwt_wt_serialize add the device
// context.  Byte layouts: sdsl_format.hpp (PARITY UNPINNED -- sdsl-lite is an
// empty submodule here and no reference-written file exists).
#include <memory>
#include <string>
#include <vector>

#include "mbrwt_internal.hpp"
#include "sdsl_format.hpp"
#include "../../include/mbrwt_wt.h"

struct mbrwt_binrel {
    std::vector<uint64_t> offsets;
    std::vector<uint32_t> cols;
    mbrwt_binrel_desc desc{};
    void finish() {
        desc.num_rows = offsets.size() - 1;
        desc.offsets = offsets.data();
        desc.cols = cols.data();
    }
};

namespace {

using mbrwt::set_error;
namespace fmt = mbrwt::fmt;

int write_stream(const mbrwt_binrel_desc &d, uint8_t *buf, uint64_t cap, uint64_t *needed) {
    if (d.num_rows && (!d.offsets || (d.offsets[d.num_rows] && !d.cols))) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    const uint64_t nrel = d.num_rows ? d.offsets[d.num_rows] : 0;
    std::vector<uint64_t> seq(nrel);
    std::vector<uint64_t> delim((1 + nrel + d.num_rows + 63) / 64, 0);
    uint64_t bit = 0;
    delim[0] |= 1;
    ++bit;
    for (uint64_t r = 0; r < d.num_rows; ++r) {
        if (d.offsets[r + 1] < d.offsets[r] || d.offsets[r + 1] > nrel) {
            set_error("offsets not ascending");
            return MBRWT_ERR_INVALID;
        }
        for (uint64_t k = d.offsets[r]; k < d.offsets[r + 1]; ++k) {
            if (d.cols[k] >= d.num_columns) {
                set_error("column id out of range");
                return MBRWT_ERR_RANGE;
            }
            seq[k] = d.cols[k];
            ++bit;  // a 0 per id
        }
        delim[bit >> 6] |= 1ull << (bit & 63);
        ++bit;
    }
    fmt::Writer w;
    fmt::put_number(w, d.num_columns);
    fmt::put_wt_int(w, seq);
    fmt::put_rrr(w, delim, bit);
    if (needed) *needed = w.buf.size();
    if (!buf || cap < w.buf.size()) {
        set_error("buffer too small");
        return MBRWT_ERR_CAPACITY;
    }
    std::memcpy(buf, w.buf.data(), w.buf.size());
    return MBRWT_OK;
}

}  // namespace

extern "C" {

int mbrwt_wt_parse(const uint8_t *bytes, uint64_t len, uint64_t *consumed, mbrwt_binrel **out) {
    if (!out || (!bytes && len)) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    *out = nullptr;
    try {
        fmt::Reader r(bytes, len);
        auto b = std::make_unique<mbrwt_binrel>();
        b->desc.num_columns = fmt::get_number(r);
        const std::vector<uint64_t> seq = fmt::get_wt_int(r);
        uint64_t dbits = 0;
        const std::vector<uint64_t> delim = fmt::get_rrr(r, &dbits);
        auto at = [&](uint64_t i) { return (delim[i >> 6] >> (i & 63)) & 1; };
        if (dbits == 0 || !at(0) || !at(dbits - 1)) throw fmt::FormatError("delimiters must start and end with 1");
        b->offsets.push_back(0);
        uint64_t k = 0;
        for (uint64_t i = 1; i < dbits; ++i) {
            if (at(i)) {
                b->offsets.push_back(k);
            } else {
                if (k >= seq.size()) throw fmt::FormatError("more delimiter zeros than symbols");
                if (seq[k] >= b->desc.num_columns) throw fmt::FormatError("symbol >= num_columns");
                b->cols.push_back((uint32_t)seq[k]);
                ++k;
            }
        }
        if (k != seq.size()) throw fmt::FormatError("symbols without delimiter zeros");
        b->finish();
        if (consumed) *consumed = r.pos;
        *out = b.release();
        return MBRWT_OK;
    } catch (const std::bad_alloc &) {
        set_error("out of host memory");
        return MBRWT_ERR_NOMEM;
    } catch (const std::exception &e) {
        set_error(std::string("BinRelWT stream: ") + e.what());
        return MBRWT_ERR_INVALID;
    }
}

const mbrwt_binrel_desc *mbrwt_binrel_get_desc(const mbrwt_binrel *b) { return b ? &b->desc : nullptr; }
void mbrwt_binrel_free(mbrwt_binrel *b) { delete b; }

int mbrwt_wt_serialize_desc(const mbrwt_binrel_desc *desc, uint8_t *buf, uint64_t cap, uint64_t *needed) {
    if (!desc) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    try {
        return write_stream(*desc, buf, cap, needed);
    } catch (const std::bad_alloc &) {
        set_error("out of host memory");
        return MBRWT_ERR_NOMEM;
    }
}

int mbrwt_wt_load(const uint8_t *bytes, uint64_t len, uint64_t *consumed, int device, mbrwt_wt **out) {
    if (!out) {
        set_error("null output pointer");
        return MBRWT_ERR_INVALID;
    }
    *out = nullptr;
    mbrwt_binrel *b = nullptr;
    int rc = mbrwt_wt_parse(bytes, len, consumed, &b);
    if (rc) return rc;
    rc = mbrwt_wt_create(&b->desc, device, out);
    mbrwt_binrel_free(b);
    return rc;
}

int mbrwt_wt_serialize(mbrwt_wt *ctx, uint8_t *buf, uint64_t cap, uint64_t *needed) {
    if (!ctx) {
        set_error("invalid argument");
        return MBRWT_ERR_INVALID;
    }
    try {
        mbrwt_binrel b;
        const uint64_t n = mbrwt_wt_num_rows(ctx);
        b.desc.num_columns = mbrwt_wt_num_columns(ctx);
        std::vector<uint64_t> rows(n);
        for (uint64_t i = 0; i < n; ++i) rows[i] = i;
        b.offsets.assign(n + 1, 0);
        b.cols.resize(mbrwt_wt_num_relations(ctx) + 1);
        uint64_t need = 0;
        if (n) {
            const int rc =
                mbrwt_wt_get_rows(ctx, rows.data(), n, b.offsets.data(), b.cols.data(), b.cols.size(), &need);
            if (rc) return rc;
        }
        b.cols.resize(need);
        b.finish();
        return write_stream(b.desc, buf, cap, needed);
    } catch (const std::bad_alloc &) {
        set_error("out of host memory");
        return MBRWT_ERR_NOMEM;
    }
}

}  // extern "C"

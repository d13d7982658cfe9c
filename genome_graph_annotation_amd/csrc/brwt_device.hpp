// brwt_device.hpp -- C++ host mirror of the reference's BinaryMatrix surface
// over the HIP engine (header-only, depends only on include/mbrwt.h).
//
// Reference interface restated (ratschlab/genome_graph_annotation):
//   class BinaryMatrix           common/binary_matrix.hpp:9-29
//   class BRWT : BinaryMatrix    annotation/hierarchical_annotation/BRWT.hpp:18-61
// BRWTDevice keeps the reference's names, argument meaning and error
// behaviour (out-of-range rows: the reference asserts, BRWT.cpp:27; here
// std::out_of_range) and adds the batched get_rows() that the device path
// is built for.  A reference build would register it where BRWTCompressed is
// selected (main.cpp:222-225); see INTEGRATION.md.
#pragma once

#include <algorithm>
#include <cstdint>
#include <fstream>
#include <istream>
#include <iterator>
#include <memory>
#include <ostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/mbrwt.h"

// Built inside the reference tree, define
// MBRWT_WITH_REFERENCE_BINARY_MATRIX and put the reference's common/ on the
// include path: BRWTDevice then derives from the reference's own BinaryMatrix.
#ifdef MBRWT_WITH_REFERENCE_BINARY_MATRIX
#include "binary_matrix.hpp"
namespace mbrwt_host {
typedef ::BinaryMatrix ReferenceBinaryMatrix;
}
#else
namespace mbrwt_host {
// common/binary_matrix.hpp:9-29, restated (the reference header pulls in
// sdsl-lite, which this image lacks)
class ReferenceBinaryMatrix {
  public:
    typedef uint64_t Row;
    typedef uint64_t Column;

    virtual ~ReferenceBinaryMatrix() {}

    virtual uint64_t num_columns() const = 0;
    virtual uint64_t num_rows() const = 0;

    // row is in [0, num_rows), column is in [0, num_columns)
    virtual bool get(Row row, Column column) const = 0;
    virtual std::vector<Column> get_row(Row row) const = 0;
    virtual std::vector<Row> get_column(Column column) const = 0;

    virtual bool load(std::istream &in) = 0;
    virtual void serialize(std::ostream &out) const = 0;

    // number of ones in the matrix
    virtual uint64_t num_relations() const = 0;
};
}  // namespace mbrwt_host
#endif

namespace mbrwt_host {

// The reference's BinaryMatrix plus the batched entry points the device path
// is built for; every other scheme keeps the defaults (a loop over get_row,
// or "not offered" so the annotator answers read by read).
class BinaryMatrix : public ReferenceBinaryMatrix {
  public:
    typedef uint64_t Row;
    typedef uint64_t Column;

    // Batched get_row: the default loops over get_row (every scheme of the
    // reference); device-backed matrices override it with one launch.
    virtual std::vector<std::vector<Column>> get_rows(const std::vector<Row> &rows) const {
        std::vector<std::vector<Column>> out;
        out.reserve(rows.size());
        for (Row r : rows) out.push_back(this->get_row(r));
        return out;
    }

    // Batched classify on the device (get_labels / get_top_labels for many
    // reads, CSR over reads); false = not offered by this scheme, and the
    // annotator answers read by read
    virtual bool labels_batch_csr(const std::vector<Row> &, const std::vector<uint64_t> &, double,
                                  std::vector<uint64_t> *, std::vector<uint32_t> *) const {
        return false;
    }
    virtual bool top_labels_batch_csr(const std::vector<Row> &, const std::vector<uint64_t> &, uint64_t,
                                      std::vector<uint64_t> *, std::vector<uint32_t> *,
                                      std::vector<uint64_t> *) const {
        return false;
    }
};

// Reads the rest of `in` into memory for a C-ABI parser and, once the parser
// has reported how many bytes it used, leaves the stream right after them --
// where the reference's stream-based load would have left it.
template <class Parse>
bool load_from_stream(std::istream &in, Parse &&parse) {
    if (!in.good()) return false;
    const std::streampos start = in.tellg();
    std::vector<char> buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    uint64_t used = 0;
    if (!parse(reinterpret_cast<const uint8_t *>(buf.data()), (uint64_t)buf.size(), &used)) return false;
    in.clear();
    if (start != std::streampos(-1)) in.seekg(start + std::streamoff(used));
    return in.good();
}

class MBRWTException : public std::runtime_error {
  public:
    MBRWTException(int status, const std::string &where)
        : std::runtime_error(where + ": " + mbrwt_strerror(status) + " (" + mbrwt_last_error_message() + ")"),
          status_(status) {}
    int status() const { return status_; }

  private:
    int status_;
};

inline void check_status(int status, const char *where) {
    if (status == MBRWT_OK) return;
    if (status == MBRWT_ERR_RANGE) throw std::out_of_range(std::string(where) + ": row or column out of range");
    throw MBRWTException(status, where);
}

// A BRWT whose queries run on an MI355X (the reference's BRWT::get_row /
// BRWT::get, BRWT.cpp:9-53).
class BRWTDevice : public BinaryMatrix {
  public:
    BRWTDevice() = default;  // the empty BRWT() (test_BRWT.cpp:15-19)

    explicit BRWTDevice(int device) : device_(device) {}

    BRWTDevice(const mbrwt_tree_desc &desc, int device = 0) : device_(device) {
        mbrwt_ctx *c = nullptr;
        check_status(mbrwt_create(&desc, device, &c), "mbrwt_create");
        ctx_.reset(c, Deleter());
    }

    static BRWTDevice synthetic(const mbrwt_synth_desc &desc, int device = 0) {
        BRWTDevice m(device);
        mbrwt_ctx *c = nullptr;
        check_status(mbrwt_create_synthetic(&desc, device, &c), "mbrwt_create_synthetic");
        m.ctx_.reset(c, Deleter());
        return m;
    }

    // BRWTBottomUpBuilder::build(columns, get_basic_partitioner(arity))
    // (BRWT_builders.cpp:20-31, :119-163), run on the device; columns[j] =
    // ceil(num_rows/64) LSB-first words.  relax_max_arity > 1 then applies
    // BRWTOptimizer::relax (:166-297) with that arity limit
    static BRWTDevice build_bottom_up(const std::vector<std::vector<uint64_t>> &columns, uint64_t num_rows,
                                      uint32_t arity, int device = 0, uint64_t relax_max_arity = 0) {
        std::vector<const uint64_t *> ptrs(columns.size());
        for (size_t j = 0; j < columns.size(); ++j) ptrs[j] = columns[j].data();
        mbrwt_columns_desc d{num_rows, columns.size(), ptrs.data(), arity};
        BRWTDevice m(device);
        mbrwt_ctx *c = nullptr;
        check_status(mbrwt_create_from_columns_relaxed(&d, relax_max_arity, device, &c),
                     "mbrwt_create_from_columns_relaxed");
        m.ctx_.reset(c, Deleter());
        return m;
    }

    // BRWTBottomUpBuilder::build with binary_grouping_greedy
    // (partitionings.cpp:148-196; `transform_anno --greedy`), then relax --
    // the reference's production build (scripts/kingsford/convert.sh:24)
    static BRWTDevice build_greedy(const std::vector<std::vector<uint64_t>> &columns, uint64_t num_rows,
                                   int device = 0, uint64_t relax_max_arity = 0) {
        int64_t prev = MBRWT_PARTITIONER_BASIC;
        check_status(mbrwt_get_build_option(MBRWT_BUILD_PARTITIONER, &prev), "build option");
        check_status(mbrwt_set_build_option(MBRWT_BUILD_PARTITIONER, MBRWT_PARTITIONER_GREEDY), "build option");
        struct Restore {  // the caller's own setting, not a fixed value
            int64_t v;
            ~Restore() { (void)mbrwt_set_build_option(MBRWT_BUILD_PARTITIONER, v); }
        } restore_{prev};
        return build_bottom_up(columns, num_rows, 2, device, relax_max_arity);
    }

    // a query handle over the same device image (mbrwt_ctx_clone): one per
    // server worker thread, so their get_rows calls do not serialise on a
    // shared workspace (the reference shares its annotator by reference
    // across the server's thread pool)
    BRWTDevice clone() const {
        if (!ctx_) return BRWTDevice(device_);
        BRWTDevice m(device_);
        mbrwt_ctx *c = nullptr;
        check_status(mbrwt_ctx_clone(ctx_.get(), &c), "mbrwt_ctx_clone");
        m.ctx_.reset(c, Deleter());
        return m;
    }

    // BRWTOptimizer::relax(brwt, max_arity) of an exported tree
    // (`annograph relax_brwt`, main.cpp:746)
    static BRWTDevice relaxed(const mbrwt_tree_desc &desc, uint64_t max_arity, int device = 0) {
        BRWTDevice m(device);
        mbrwt_ctx *c = nullptr;
        check_status(mbrwt_create_relaxed(&desc, max_arity, device, &c), "mbrwt_create_relaxed");
        m.ctx_.reset(c, Deleter());
        return m;
    }

    uint64_t num_columns() const override { return ctx_ ? mbrwt_num_columns(ctx_.get()) : 0; }
    uint64_t num_rows() const override { return ctx_ ? mbrwt_num_rows(ctx_.get()) : 0; }
    uint64_t num_relations() const override { return ctx_ ? mbrwt_num_relations(ctx_.get()) : 0; }
    uint64_t num_nodes() const { return ctx_ ? mbrwt_num_nodes(ctx_.get()) : 1; }

    bool get(Row row, Column column) const override {
        if (!ctx_) throw std::out_of_range("get on an empty BRWT");
        uint8_t out = 0;
        check_status(mbrwt_get_batch(ctx_.get(), &row, &column, 1, &out), "BRWTDevice::get");
        return out != 0;
    }

    std::vector<Column> get_row(Row row) const override { return get_rows({row}).at(0); }

    // BRWT::get_column (BRWT.cpp:55-85): ascending rows of the column
    std::vector<Row> get_column(Column column) const override {
        if (!ctx_) throw std::out_of_range("get_column on an empty BRWT");
        uint64_t need = 0;
        int st = mbrwt_get_column(ctx_.get(), column, nullptr, 0, &need);
        std::vector<Row> rows;
        if (st == MBRWT_OK) return rows;  // empty column
        if (st != MBRWT_ERR_CAPACITY) check_status(st, "BRWTDevice::get_column");
        rows.resize(need);
        check_status(mbrwt_get_column(ctx_.get(), column, rows.data(), rows.size(), &need), "BRWTDevice::get_column");
        rows.resize(need);
        return rows;
    }

    std::vector<std::vector<Column>> get_rows(const std::vector<Row> &rows) const override {
        std::vector<uint64_t> offsets;
        std::vector<uint32_t> cols;
        get_rows_csr(rows, &offsets, &cols);
        std::vector<std::vector<Column>> out(rows.size());
        for (size_t i = 0; i < rows.size(); ++i) out[i].assign(cols.begin() + offsets[i], cols.begin() + offsets[i + 1]);
        return out;
    }

    // StaticBinRelAnnotator::get_labels(indices, presence_ratio)
    // (annotate_static.cpp:71-94) for many reads in one call: read r =
    // rows[read_offsets[r] .. read_offsets[r+1]); label_offsets[reads+1] and
    // the ascending label codes of each read (mbrwt_get_labels_batch)
    void get_labels_batch_csr(const std::vector<Row> &rows, const std::vector<uint64_t> &read_offsets,
                              double presence_ratio, std::vector<uint64_t> *label_offsets,
                              std::vector<uint32_t> *labels) const {
        if (read_offsets.empty()) throw std::invalid_argument("read_offsets needs n_reads + 1 entries");
        const uint64_t n_reads = read_offsets.size() - 1;
        label_offsets->assign(read_offsets.size(), 0);
        labels->clear();
        if (!ctx_) {
            if (!rows.empty()) throw std::out_of_range("get_labels on an empty BRWT");
            return;
        }
        uint64_t cap = std::max<uint64_t>(16, 4 * rows.size()), need = 0;
        for (;;) {
            labels->resize(cap);
            int st = mbrwt_get_labels_batch(ctx_.get(), rows.data(), rows.size(), read_offsets.data(), n_reads,
                                            presence_ratio, label_offsets->data(), labels->data(), cap, &need);
            if (st == MBRWT_ERR_CAPACITY) {
                cap = need;
                continue;
            }
            check_status(st, "BRWTDevice::get_labels_batch");
            labels->resize(need);
            return;
        }
    }

    // MultiLabelEncoded::get_top_labels(indices, num_top) (annotate.cpp:57-83)
    // for many reads in one call (mbrwt_get_top_labels_batch): per read, the
    // label codes and their counts by count descending (ties: code ascending)
    void get_top_labels_batch_csr(const std::vector<Row> &rows, const std::vector<uint64_t> &read_offsets,
                                  uint64_t num_top, std::vector<uint64_t> *label_offsets,
                                  std::vector<uint32_t> *labels, std::vector<uint64_t> *counts) const {
        if (read_offsets.empty()) throw std::invalid_argument("read_offsets needs n_reads + 1 entries");
        const uint64_t n_reads = read_offsets.size() - 1;
        label_offsets->assign(read_offsets.size(), 0);
        labels->clear();
        counts->clear();
        if (!ctx_) {
            if (!rows.empty()) throw std::out_of_range("get_top_labels on an empty BRWT");
            return;
        }
        uint64_t cap = std::max<uint64_t>(16, 4 * rows.size()), need = 0;
        for (;;) {
            labels->resize(cap);
            counts->resize(cap);
            int st = mbrwt_get_top_labels_batch(ctx_.get(), rows.data(), rows.size(), read_offsets.data(), n_reads,
                                                num_top, label_offsets->data(), labels->data(), counts->data(), cap,
                                                &need);
            if (st == MBRWT_ERR_CAPACITY) {
                cap = need;
                continue;
            }
            check_status(st, "BRWTDevice::get_top_labels_batch");
            labels->resize(need);
            counts->resize(need);
            return;
        }
    }

    bool labels_batch_csr(const std::vector<Row> &rows, const std::vector<uint64_t> &read_offsets, double ratio,
                          std::vector<uint64_t> *lab_off, std::vector<uint32_t> *labels) const override {
        // MBRWT_ERR_UNSUPPORTED (more columns than the device histogram holds):
        // the annotator falls back to per-read count_labels, as the reference
        // has no column limit there
        try {
            get_labels_batch_csr(rows, read_offsets, ratio, lab_off, labels);
        } catch (const MBRWTException &e) {
            if (e.status() == MBRWT_ERR_UNSUPPORTED) return false;
            throw;
        }
        return true;
    }
    bool top_labels_batch_csr(const std::vector<Row> &rows, const std::vector<uint64_t> &read_offsets,
                              uint64_t num_top, std::vector<uint64_t> *lab_off, std::vector<uint32_t> *labels,
                              std::vector<uint64_t> *counts) const override {
        try {
            get_top_labels_batch_csr(rows, read_offsets, num_top, lab_off, labels, counts);
        } catch (const MBRWTException &e) {
            if (e.status() == MBRWT_ERR_UNSUPPORTED) return false;  // per-read fallback
            throw;
        }
        return true;
    }

    // CSR form: offsets[rows.size()+1], cols in the reference's per-row order
    void get_rows_csr(const std::vector<Row> &rows, std::vector<uint64_t> *offsets,
                      std::vector<uint32_t> *cols) const {
        if (!ctx_) {
            if (!rows.empty()) throw std::out_of_range("get_row on an empty BRWT");
            offsets->assign(1, 0);
            cols->clear();
            return;
        }
        offsets->assign(rows.size() + 1, 0);
        uint64_t cap = std::max<uint64_t>(16, 16 * rows.size()), need = 0;
        for (;;) {
            cols->resize(cap);
            int st = mbrwt_get_rows(ctx_.get(), rows.data(), rows.size(), offsets->data(), cols->data(), cap, &need);
            if (st == MBRWT_ERR_CAPACITY) {
                cap = need;
                continue;
            }
            check_status(st, "BRWTDevice::get_rows");
            cols->resize(need);
            return;
        }
    }

    // BRWT::load (BRWT.cpp:87-111): the BRWT stream at the stream's position
    // (mbrwt_load); false on a bad stream, like the reference
    bool load(std::istream &in) override {
        try {
            return load_from_stream(in, [&](const uint8_t *p, uint64_t n, uint64_t *used) {
                mbrwt_ctx *c = nullptr;
                if (mbrwt_load(p, n, used, device_, &c) != MBRWT_OK) return false;
                ctx_.reset(c, Deleter());
                return true;
            });
        } catch (...) {
            return false;
        }
    }

    // BRWT::serialize (BRWT.cpp:113-128): the device image read back
    // (mbrwt_tree_export) and written in the reference's stream format
    void serialize(std::ostream &out) const override {
        if (!out.good()) throw std::ofstream::failure("Error when dumping BRWT");
        std::vector<uint8_t> bytes;
        mbrwt_tree *t = nullptr;
        mbrwt_tree_desc empty{};
        if (ctx_) check_status(mbrwt_tree_export(ctx_.get(), &t), "BRWTDevice::serialize");
        std::unique_ptr<mbrwt_tree, void (*)(mbrwt_tree *)> hold(t, mbrwt_tree_free);
        const mbrwt_tree_desc *d = t ? mbrwt_tree_get_desc(t) : &empty;
        uint64_t need = 0;
        int st = mbrwt_tree_serialize(d, nullptr, 0, &need);
        if (st != MBRWT_ERR_CAPACITY) check_status(st, "BRWTDevice::serialize");
        bytes.resize(need);
        check_status(mbrwt_tree_serialize(d, bytes.data(), bytes.size(), &need), "BRWTDevice::serialize");
        out.write(reinterpret_cast<const char *>(bytes.data()), (std::streamsize)bytes.size());
    }

    mbrwt_ctx *handle() const { return ctx_.get(); }
    int device() const { return device_; }

  private:
    struct Deleter {
        void operator()(mbrwt_ctx *c) const { mbrwt_destroy(c); }
    };
    std::shared_ptr<mbrwt_ctx> ctx_{nullptr, Deleter()};
    int device_ = 0;

  public:
    BRWTDevice(const BRWTDevice &) = default;
    BRWTDevice &operator=(const BRWTDevice &) = default;
};

// A BRWT replicated on several GPUs of one process (mbrwt_multi_*): get_rows
// batches are cut into one contiguous slice per replica and reassembled into
// one CSR; point and column queries and serialisation use replica 0.  The
// reference's `annograph classify` (one process, a ThreadPool,
// main.cpp:462-497) runs StaticBinRelAnnotator<BRWTMultiDevice> to use every
// GPU of the node.
class BRWTMultiDevice : public BinaryMatrix {
  public:
    BRWTMultiDevice() = default;
    BRWTMultiDevice(const mbrwt_tree_desc &desc, const std::vector<int> &devices) {
        mbrwt_multi *m = nullptr;
        check_status(mbrwt_multi_create(&desc, devices.data(), (int)devices.size(), &m), "mbrwt_multi_create");
        m_.reset(m, Deleter());
    }
    static BRWTMultiDevice synthetic(const mbrwt_synth_desc &desc, const std::vector<int> &devices) {
        BRWTMultiDevice x;
        mbrwt_multi *m = nullptr;
        check_status(mbrwt_multi_create_synthetic(&desc, devices.data(), (int)devices.size(), &m),
                     "mbrwt_multi_create_synthetic");
        x.m_.reset(m, Deleter());
        return x;
    }
    explicit BRWTMultiDevice(const std::vector<int> &devices) : devices_(devices) {}

    int replicas() const { return m_ ? mbrwt_multi_size(m_.get()) : 0; }

    uint64_t num_columns() const override { return m_ ? mbrwt_num_columns(r0()) : 0; }
    uint64_t num_rows() const override { return m_ ? mbrwt_num_rows(r0()) : 0; }
    uint64_t num_relations() const override { return m_ ? mbrwt_num_relations(r0()) : 0; }

    bool get(Row row, Column column) const override {
        if (!m_) throw std::out_of_range("get on an empty BRWT");
        uint8_t out = 0;
        check_status(mbrwt_get_batch(r0(), &row, &column, 1, &out), "BRWTMultiDevice::get");
        return out != 0;
    }
    std::vector<Column> get_row(Row row) const override { return get_rows({row}).at(0); }
    std::vector<Row> get_column(Column column) const override {
        if (!m_) throw std::out_of_range("get_column on an empty BRWT");
        uint64_t need = 0;
        int st = mbrwt_get_column(r0(), column, nullptr, 0, &need);
        std::vector<Row> rows;
        if (st == MBRWT_OK) return rows;
        if (st != MBRWT_ERR_CAPACITY) check_status(st, "BRWTMultiDevice::get_column");
        rows.resize(need);
        check_status(mbrwt_get_column(r0(), column, rows.data(), rows.size(), &need), "BRWTMultiDevice::get_column");
        rows.resize(need);
        return rows;
    }
    std::vector<std::vector<Column>> get_rows(const std::vector<Row> &rows) const override {
        std::vector<uint64_t> offsets;
        std::vector<uint32_t> cols;
        get_rows_csr(rows, &offsets, &cols);
        std::vector<std::vector<Column>> out(rows.size());
        for (size_t i = 0; i < rows.size(); ++i) out[i].assign(cols.begin() + offsets[i], cols.begin() + offsets[i + 1]);
        return out;
    }
    void get_rows_csr(const std::vector<Row> &rows, std::vector<uint64_t> *offsets, std::vector<uint32_t> *cols) const {
        if (!m_) {
            if (!rows.empty()) throw std::out_of_range("get_row on an empty BRWT");
            offsets->assign(1, 0);
            cols->clear();
            return;
        }
        offsets->assign(rows.size() + 1, 0);
        uint64_t cap = std::max<uint64_t>(16, 16 * rows.size()), need = 0;
        for (;;) {
            cols->resize(cap);
            int st = mbrwt_multi_get_rows(m_.get(), rows.data(), rows.size(), offsets->data(), cols->data(), cap, &need);
            if (st == MBRWT_ERR_CAPACITY) {
                cap = need;
                continue;
            }
            check_status(st, "BRWTMultiDevice::get_rows");
            cols->resize(need);
            return;
        }
    }
    // BRWT::load onto every replica (mbrwt_multi_load); false on a bad stream
    bool load(std::istream &in) override {
        try {
            return load_from_stream(in, [&](const uint8_t *p, uint64_t n, uint64_t *used) {
                mbrwt_multi *m = nullptr;
                const std::vector<int> devs = devices_.empty() ? std::vector<int>{0} : devices_;
                if (mbrwt_multi_load(p, n, used, devs.data(), (int)devs.size(), &m) != MBRWT_OK) return false;
                m_.reset(m, Deleter());
                return true;
            });
        } catch (...) {
            return false;
        }
    }
    void serialize(std::ostream &out) const override {
        if (!out.good()) throw std::ofstream::failure("Error when dumping BRWT");
        mbrwt_tree *t = nullptr;
        mbrwt_tree_desc empty{};
        if (m_) check_status(mbrwt_tree_export(r0(), &t), "BRWTMultiDevice::serialize");
        std::unique_ptr<mbrwt_tree, void (*)(mbrwt_tree *)> hold(t, mbrwt_tree_free);
        const mbrwt_tree_desc *d = t ? mbrwt_tree_get_desc(t) : &empty;
        uint64_t need = 0;
        int st = mbrwt_tree_serialize(d, nullptr, 0, &need);
        if (st != MBRWT_ERR_CAPACITY) check_status(st, "BRWTMultiDevice::serialize");
        std::vector<uint8_t> bytes(need);
        check_status(mbrwt_tree_serialize(d, bytes.data(), bytes.size(), &need), "BRWTMultiDevice::serialize");
        out.write(reinterpret_cast<const char *>(bytes.data()), (std::streamsize)bytes.size());
    }

  private:
    mbrwt_ctx *r0() const { return mbrwt_multi_replica(m_.get(), 0); }
    struct Deleter {
        void operator()(mbrwt_multi *m) const { mbrwt_multi_destroy(m); }
    };
    std::shared_ptr<mbrwt_multi> m_{nullptr, Deleter()};
    std::vector<int> devices_;
};

}  // namespace mbrwt_host

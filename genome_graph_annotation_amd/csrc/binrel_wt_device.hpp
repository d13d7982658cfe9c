// binrel_wt_device.hpp -- C++ host mirror of BinRelWT_sdsl over the device
// engine (header-only, depends only on include/mbrwt_wt.h).
//
// Reference interface restated: class BinRelWT_sdsl : BinaryMatrix
// (annotation/bin_rel_wt/bin_rel_wt_sdsl.hpp:9-43).  Constructed from the
// rows generate_rows would emit (bin_rel_wt_sdsl.cpp:10-40); queries go to
// the HIP wavelet-matrix kernels.  Out-of-range rows/columns (asserts / UB in
// the reference) throw std::out_of_range.
#pragma once

#include <fstream>
#include <functional>
#include <iterator>

#include "../../include/mbrwt_wt.h"
#include "brwt_device.hpp"

namespace mbrwt_host {

class BinRelWTDevice : public BinaryMatrix {
  public:
    typedef std::vector<Column> RowSetBits;
    typedef std::function<void(const RowSetBits &)> RowCallback;

    BinRelWTDevice() = default;  // BinRelWT_sdsl(): no rows, no columns

    // bin_rel_wt_sdsl.cpp:10-40 (num_relations is only a capacity hint here)
    BinRelWTDevice(const std::function<void(const RowCallback &)> &generate_rows, uint64_t num_relations,
                   uint64_t num_columns, int device = 0) {
        std::vector<uint64_t> offsets{0};
        std::vector<uint32_t> cols;
        cols.reserve(num_relations);
        generate_rows([&](const RowSetBits &row) {
            for (auto c : row) cols.push_back((uint32_t)c);
            offsets.push_back(cols.size());
        });
        mbrwt_binrel_desc d{offsets.size() - 1, num_columns, offsets.data(), cols.data()};
        mbrwt_wt *c = nullptr;
        check_status(mbrwt_wt_create(&d, device, &c), "mbrwt_wt_create");
        ctx_.reset(c, Deleter());
    }

    static BinRelWTDevice synthetic(const mbrwt_binrel_synth_desc &desc, int device = 0) {
        BinRelWTDevice m;
        mbrwt_wt *c = nullptr;
        check_status(mbrwt_wt_create_synthetic(&desc, device, &c), "mbrwt_wt_create_synthetic");
        m.ctx_.reset(c, Deleter());
        return m;
    }

    uint64_t num_columns() const override { return ctx_ ? mbrwt_wt_num_columns(ctx_.get()) : 0; }
    uint64_t num_rows() const override { return ctx_ ? mbrwt_wt_num_rows(ctx_.get()) : 0; }
    uint64_t num_relations() const override { return ctx_ ? mbrwt_wt_num_relations(ctx_.get()) : 0; }

    bool get(Row row, Column column) const override {
        if (!ctx_) throw std::out_of_range("get on an empty BinRelWT");
        uint8_t out = 0;
        check_status(mbrwt_wt_get_batch(ctx_.get(), &row, &column, 1, &out), "BinRelWTDevice::get");
        return out != 0;
    }

    std::vector<Column> get_row(Row row) const override { return get_rows({row}).at(0); }

    std::vector<std::vector<Column>> get_rows(const std::vector<Row> &rows) const override {
        if (!ctx_) {
            if (!rows.empty()) throw std::out_of_range("get_row on an empty BinRelWT");
            return {};
        }
        std::vector<uint64_t> offsets(rows.size() + 1, 0);
        std::vector<uint32_t> cols;
        uint64_t need = 0;
        int st = mbrwt_wt_get_rows(ctx_.get(), rows.data(), rows.size(), offsets.data(), nullptr, 0, &need);
        if (st == MBRWT_ERR_CAPACITY) {
            cols.resize(need);
            st = mbrwt_wt_get_rows(ctx_.get(), rows.data(), rows.size(), offsets.data(), cols.data(), cols.size(),
                                   &need);
        }
        check_status(st, "BinRelWTDevice::get_rows");
        std::vector<std::vector<Column>> out(rows.size());
        for (size_t i = 0; i < rows.size(); ++i) out[i].assign(cols.begin() + offsets[i], cols.begin() + offsets[i + 1]);
        return out;
    }

    // batched classify (include/mbrwt_wt.h mbrwt_wt_get[_top]_labels_batch)
    bool labels_batch_csr(const std::vector<Row> &rows, const std::vector<uint64_t> &read_offsets, double ratio,
                          std::vector<uint64_t> *lab_off, std::vector<uint32_t> *labels) const override {
        if (read_offsets.empty()) throw std::invalid_argument("read_offsets needs n_reads + 1 entries");
        lab_off->assign(read_offsets.size(), 0);
        labels->clear();
        if (!ctx_) {
            if (!rows.empty()) throw std::out_of_range("get_labels on an empty BinRelWT");
            return true;
        }
        uint64_t cap = std::max<uint64_t>(16, 4 * rows.size()), need = 0;
        for (;;) {
            labels->resize(cap);
            int st = mbrwt_wt_get_labels_batch(ctx_.get(), rows.data(), rows.size(), read_offsets.data(),
                                               read_offsets.size() - 1, ratio, lab_off->data(), labels->data(), cap,
                                               &need);
            if (st == MBRWT_ERR_CAPACITY) {
                cap = need;
                continue;
            }
            if (st == MBRWT_ERR_UNSUPPORTED) return false;  // per-read count_labels fallback
            check_status(st, "BinRelWTDevice::get_labels_batch");
            labels->resize(need);
            return true;
        }
    }
    bool top_labels_batch_csr(const std::vector<Row> &rows, const std::vector<uint64_t> &read_offsets,
                              uint64_t num_top, std::vector<uint64_t> *lab_off, std::vector<uint32_t> *labels,
                              std::vector<uint64_t> *counts) const override {
        if (read_offsets.empty()) throw std::invalid_argument("read_offsets needs n_reads + 1 entries");
        lab_off->assign(read_offsets.size(), 0);
        labels->clear();
        counts->clear();
        if (!ctx_) {
            if (!rows.empty()) throw std::out_of_range("get_top_labels on an empty BinRelWT");
            return true;
        }
        uint64_t cap = std::max<uint64_t>(16, 4 * rows.size()), need = 0;
        for (;;) {
            labels->resize(cap);
            counts->resize(cap);
            int st = mbrwt_wt_get_top_labels_batch(ctx_.get(), rows.data(), rows.size(), read_offsets.data(),
                                                   read_offsets.size() - 1, num_top, lab_off->data(), labels->data(),
                                                   counts->data(), cap, &need);
            if (st == MBRWT_ERR_CAPACITY) {
                cap = need;
                continue;
            }
            if (st == MBRWT_ERR_UNSUPPORTED) return false;  // per-read count_labels fallback
            check_status(st, "BinRelWTDevice::get_top_labels_batch");
            labels->resize(need);
            counts->resize(need);
            return true;
        }
    }

    std::vector<Row> get_column(Column column) const override {
        if (!ctx_) throw std::out_of_range("get_column on an empty BinRelWT");
        uint64_t need = 0;
        int st = mbrwt_wt_get_column(ctx_.get(), column, nullptr, 0, &need);
        std::vector<Row> rows;
        if (st == MBRWT_OK) return rows;
        if (st != MBRWT_ERR_CAPACITY) check_status(st, "BinRelWTDevice::get_column");
        rows.resize(need);
        check_status(mbrwt_wt_get_column(ctx_.get(), column, rows.data(), rows.size(), &need),
                     "BinRelWTDevice::get_column");
        rows.resize(need);
        return rows;
    }

    // BinRelWT_sdsl::load / serialize (bin_rel_wt_sdsl.cpp:113-132) through
    // mbrwt_wt_load / mbrwt_wt_serialize (include/mbrwt_wt.h; byte layout
    // parity unpinned).  load reads the rest of the stream, returns false on
    // a malformed one as the reference's does; serialize throws on a bad stream.
    bool load(std::istream &in) override {
        if (!in.good()) return false;
        const std::streampos at = in.tellg();
        std::vector<uint8_t> bytes((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
        mbrwt_binrel *b = nullptr;
        uint64_t used = 0;
        if (mbrwt_wt_parse(bytes.data(), bytes.size(), &used, &b) != MBRWT_OK) return false;
        std::unique_ptr<mbrwt_binrel, void (*)(mbrwt_binrel *)> owned(b, mbrwt_binrel_free);
        const mbrwt_binrel_desc *d = mbrwt_binrel_get_desc(b);
        if (d->num_rows == 0) {  // BinRelWT_sdsl(): the empty matrix
            ctx_.reset();
        } else {
            mbrwt_wt *c = nullptr;
            if (mbrwt_wt_create(d, 0, &c) != MBRWT_OK) return false;
            ctx_.reset(c, Deleter());
        }
        in.clear();
        if (at != std::streampos(-1)) in.seekg(at + std::streamoff(used));  // just past what was read
        return true;
    }
    void serialize(std::ostream &out) const override {
        if (!out.good()) throw std::ofstream::failure("Bad stream");
        uint64_t need = 0;
        const uint64_t zero = 0;
        const mbrwt_binrel_desc empty{0, 0, &zero, nullptr};
        auto write = [&](uint8_t *buf, uint64_t cap) {
            return ctx_ ? mbrwt_wt_serialize(ctx_.get(), buf, cap, &need)
                        : mbrwt_wt_serialize_desc(&empty, buf, cap, &need);
        };
        int st = write(nullptr, 0);
        if (st != MBRWT_ERR_CAPACITY && st != MBRWT_OK) check_status(st, "BinRelWTDevice::serialize");
        std::vector<uint8_t> buf(need);
        check_status(write(buf.data(), buf.size()), "BinRelWTDevice::serialize");
        out.write(reinterpret_cast<const char *>(buf.data()), (std::streamsize)need);
    }

  private:
    struct Deleter {
        void operator()(mbrwt_wt *c) const { mbrwt_wt_destroy(c); }
    };
    std::shared_ptr<mbrwt_wt> ctx_{nullptr, Deleter()};

};

}  // namespace mbrwt_host

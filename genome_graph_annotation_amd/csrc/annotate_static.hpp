// annotate_static.hpp -- C++ host mirror of the reference's static
// annotator over any BinaryMatrix, used with BRWTDevice for the device path.
//
// Restated interfaces (ratschlab/genome_graph_annotation):
//   AnnotationCategory, MultiLabelAnnotation  common/annotate.hpp:29-108
//   LabelEncoder<Label>                       common/annotate.hpp:110-140, annotate.cpp:12-52
//   MultiLabelEncoded (get_top_labels)        common/annotate.hpp:143-196, annotate.cpp:57-83
//   StaticBinRelAnnotator<Matrix>             annotation/annotate_static.{hpp,cpp}
//     has_label :26-33, has_labels :35-55, get_labels(i) :57-67,
//     get_labels(indices, ratio) :71-94, serialize / merge_load :96-130,
//     count_labels :149-162
// count_labels (the `classify` hot loop, annotate_static.cpp:155-159) goes
// through the matrix's batched get_rows(), i.e. one device launch for the
// whole index list instead of one get_row per index.
//
// Built inside the reference tree, define MBRWT_WITH_REFERENCE_ANNOTATE (and
// put the reference's common/ on the include path): the annotator then derives
// from the reference's own annotate::MultiLabelEncoded and uses its
// LabelEncoder, so AnnotatedDBG takes it unchanged (INTEGRATION.md §2;
// tests/test_reference_headers.py compiles exactly that).
#pragma once

#include <algorithm>
#include <cassert>
#include <cmath>
#include <fstream>
#include <iostream>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "brwt_device.hpp"

#ifdef MBRWT_WITH_REFERENCE_ANNOTATE
#include "annotate.hpp"
namespace mbrwt_host {
template <typename Label = std::string>
using LabelEncoder = ::annotate::LabelEncoder<Label>;
template <typename IndexType, typename LabelType>
using MultiLabelEncoded = ::annotate::MultiLabelEncoded<IndexType, LabelType>;
}  // namespace mbrwt_host
#else
#include "sdsl_format.hpp"
namespace mbrwt_host {

// common/annotate.hpp:29-40
template <typename Index, typename LabelType>
class AnnotationCategory {
  public:
    virtual ~AnnotationCategory() {}

    virtual LabelType get(Index i) const = 0;
    virtual void add(Index i, const LabelType &label) = 0;
    virtual void set(Index i, const LabelType &label) = 0;

    virtual void serialize(const std::string &filename) const = 0;
    virtual bool load(const std::string &filename) { return merge_load({filename}); }
    virtual bool merge_load(const std::vector<std::string> &filenames) = 0;
};

// common/annotate.hpp:46-106
template <typename IndexType, typename LabelType>
class MultiLabelAnnotation : public AnnotationCategory<IndexType, std::vector<LabelType>> {
  public:
    typedef IndexType Index;
    typedef LabelType Label;
    typedef std::vector<Label> VLabels;

    virtual ~MultiLabelAnnotation() {}

    virtual VLabels get(Index i) const override final { return get_labels(i); }
    virtual void set(Index i, const VLabels &labels) override final { set_labels(i, labels); }
    virtual void add(Index i, const VLabels &labels) override final { add_labels(i, labels); }

    virtual void set_labels(Index i, const VLabels &labels) = 0;
    virtual VLabels get_labels(Index i) const = 0;

    virtual void add_label(Index i, const Label &label) = 0;
    virtual void add_labels(Index i, const VLabels &labels) = 0;
    virtual void add_labels(const std::vector<Index> &indices, const VLabels &labels) = 0;

    virtual bool has_label(Index i, const Label &label) const = 0;
    virtual bool has_labels(Index i, const VLabels &labels) const = 0;

    virtual void serialize(const std::string &filename) const override = 0;
    virtual bool merge_load(const std::vector<std::string> &filenames) override = 0;

    virtual void insert_rows(const std::vector<Index> &rows) = 0;

    virtual VLabels get_labels(const std::vector<Index> &indices, double presence_ratio) const = 0;
    virtual std::vector<std::pair<Label, size_t>> get_top_labels(const std::vector<Index> &indices,
                                                                 size_t num_top = static_cast<size_t>(-1)) const = 0;

    virtual uint64_t num_objects() const = 0;
    virtual size_t num_labels() const = 0;
    virtual uint64_t num_relations() const = 0;
};

template <typename Label = std::string>
class LabelEncoder {
  public:
    // annotate.cpp:23-31
    size_t insert_and_encode(const Label &label) {
        auto it = encode_label_.find(label);
        if (it != encode_label_.end()) return it->second;
        encode_label_[label] = decode_label_.size();
        decode_label_.push_back(label);
        return decode_label_.size() - 1;
    }
    // annotate.cpp:12-20: throws if the label does not exist
    size_t encode(const Label &label) const {
        auto it = encode_label_.find(label);
        if (it == encode_label_.end()) throw std::runtime_error("ERROR: No such label");
        return it->second;
    }
    // annotate.hpp:128: throws on a bad code
    const Label &decode(size_t code) const { return decode_label_.at(code); }
    size_t size() const { return decode_label_.size(); }

    // annotate.cpp:33-52 (std::string labels): the label -> code map
    // (serialize_string_number_map: #entries, the keys as libmaus2 strings,
    // the codes as an int_vector<> of width 64; written here in code order,
    // the reference writes its unordered_map's order) and then the code ->
    // label vector (libmaus2 string vector).  Byte layout: sdsl_format.hpp
    // (parity unpinned).
    bool load(std::istream &instream) {
        static_assert(std::is_same<Label, std::string>::value, "LabelEncoder I/O is defined for string labels");
        try {
            std::unordered_map<Label, uint64_t> enc;
            std::vector<Label> dec;
            bool ok = load_from_stream(instream, [&](const uint8_t *p, uint64_t n, uint64_t *used) {
                mbrwt::fmt::Reader r(p, n);
                const uint64_t k = mbrwt::fmt::get_number(r);
                if (k > n) return false;
                std::vector<std::string> keys;
                for (uint64_t i = 0; i < k; ++i) keys.push_back(mbrwt::fmt::get_string(r));
                const mbrwt::fmt::IntVector vals = mbrwt::fmt::get_int_vector(r);
                if (vals.len != k) return false;
                for (uint64_t i = 0; i < k; ++i) enc.emplace(std::move(keys[i]), vals.get(i));
                dec = mbrwt::fmt::get_string_vector(r);
                *used = r.pos;
                return true;
            });
            if (!ok) return false;
            encode_label_ = std::move(enc);
            decode_label_ = std::move(dec);
            return true;
        } catch (...) {
            return false;
        }
    }
    void serialize(std::ostream &outstream) const {
        static_assert(std::is_same<Label, std::string>::value, "LabelEncoder I/O is defined for string labels");
        if (!outstream.good()) throw std::ofstream::failure("Bad stream");
        mbrwt::fmt::Writer w;
        mbrwt::fmt::put_number(w, decode_label_.size());
        mbrwt::fmt::IntVector vals(decode_label_.size(), 64);
        for (size_t i = 0; i < decode_label_.size(); ++i) {
            mbrwt::fmt::put_string(w, decode_label_[i]);
            vals.set(i, encode_label_.at(decode_label_[i]));
        }
        mbrwt::fmt::put_int_vector(w, vals);
        mbrwt::fmt::put_string_vector(w, decode_label_);
        outstream.write(reinterpret_cast<const char *>(w.buf.data()), (std::streamsize)w.buf.size());
    }

    void clear() {
        encode_label_.clear();
        decode_label_.clear();
    }

  private:
    std::unordered_map<Label, uint64_t> encode_label_;
    std::vector<Label> decode_label_;
};

// common/annotate.hpp:143-196
template <typename IndexType, typename LabelType>
class MultiLabelEncoded : public MultiLabelAnnotation<IndexType, LabelType> {
  public:
    using Index = typename MultiLabelAnnotation<IndexType, LabelType>::Index;
    using Label = typename MultiLabelAnnotation<IndexType, LabelType>::Label;
    using VLabels = typename MultiLabelAnnotation<IndexType, LabelType>::VLabels;

    virtual ~MultiLabelEncoded() {}

    // annotate.cpp:57-83 (std::sort: ties in unspecified order, as in the reference)
    virtual std::vector<std::pair<Label, size_t>> get_top_labels(
        const std::vector<Index> &indices, size_t num_top = static_cast<size_t>(-1)) const override final {
        auto counter = count_labels(indices);
        std::vector<std::pair<size_t, size_t>> counts;
        for (size_t j = 0; j < counter.size(); ++j)
            if (counter[j]) counts.emplace_back(j, counter[j]);
        std::sort(counts.begin(), counts.end(), [](const auto &a, const auto &b) { return a.second > b.second; });
        counts.resize(std::min(counts.size(), num_top));
        std::vector<std::pair<Label, size_t>> top;
        for (const auto &p : counts) top.emplace_back(label_encoder_.decode(p.first), p.second);
        return top;
    }

  protected:
    virtual std::vector<uint64_t> count_labels(const std::vector<Index> &indices) const = 0;

    LabelEncoder<Label> label_encoder_;
};

}  // namespace mbrwt_host
#endif

namespace mbrwt_host {

// file extension of a static annotator over each matrix type
// (annotation/static_annotators_def.hpp:13-17, annotate_static.cpp:11-20)
template <class Matrix>
struct AnnotatorExtension {
    static std::string value() { return ".annodbg"; }
};
template <>
struct AnnotatorExtension<BRWTDevice> {
    static std::string value() { return ".brwt.annodbg"; }  // kBRWTExtension
};
class BinRelWTDevice;
template <>
struct AnnotatorExtension<BinRelWTDevice> {
    static std::string value() { return ".bin_rel_wt_sdsl.annodbg"; }  // kBinRelWT_sdslExtension
};

// utils::remove_suffix (common/utils.cpp:179-187)
inline std::string remove_suffix(const std::string &str, const std::string &suffix) {
    const std::string actual = str.substr(std::max(0, static_cast<int>(str.size()) - static_cast<int>(suffix.size())));
    return actual == suffix ? str.substr(0, str.size() - suffix.size()) : str;
}

template <class BinaryMatrixType, typename Label = std::string>
class StaticBinRelAnnotator : public MultiLabelEncoded<uint64_t, Label> {
    using Base = MultiLabelEncoded<uint64_t, Label>;

  public:
    using Index = typename Base::Index;
    using VLabels = typename Base::VLabels;

    // annotate_static.hpp:19-21 (a default-constructed matrix, then merge_load)
    StaticBinRelAnnotator() : matrix_(make_default()) {}
    StaticBinRelAnnotator(std::unique_ptr<BinaryMatrixType> &&matrix, const LabelEncoder<Label> &label_encoder)
        : matrix_(std::move(matrix)) {
        if (!matrix_) throw std::invalid_argument("null matrix");
        this->label_encoder_ = label_encoder;
    }
    // shared form (several annotators over one device structure)
    StaticBinRelAnnotator(std::shared_ptr<BinaryMatrixType> matrix, const LabelEncoder<Label> &label_encoder)
        : matrix_(std::move(matrix)) {
        if (!matrix_) throw std::invalid_argument("null matrix");
        this->label_encoder_ = label_encoder;
    }

    // annotate_static.cpp:26-33: false on an unknown label or a failed get
    bool has_label(Index i, const Label &label) const override {
        try {
            return matrix_->get(i, this->label_encoder_.encode(label));
        } catch (...) {
            return false;
        }
    }

    // annotate_static.cpp:35-55
    bool has_labels(Index i, const VLabels &labels) const override {
        std::set<size_t> querying_codes;
        try {
            for (const auto &label : labels) querying_codes.insert(this->label_encoder_.encode(label));
        } catch (...) {
            return false;
        }
        std::set<size_t> encoded_labels;
        for (auto col : matrix_->get_row(i)) encoded_labels.insert(col);
        return std::includes(encoded_labels.begin(), encoded_labels.end(), querying_codes.begin(),
                             querying_codes.end());
    }

    // annotate_static.cpp:57-67
    VLabels get_labels(Index i) const override {
        VLabels labels;
        for (auto col : matrix_->get_row(i)) labels.push_back(this->label_encoder_.decode(col));
        return labels;
    }

    // annotate_static.cpp:71-94: labels present in at least
    // ceil(|indices| * presence_ratio) rows (any row if the ratio is 0)
    VLabels get_labels(const std::vector<Index> &indices, double presence_ratio) const override {
        assert(presence_ratio >= 0 && presence_ratio <= 1);
        const size_t min_labels_discovered =
            presence_ratio == 0 ? 1 : (size_t)std::ceil(indices.size() * presence_ratio);
        auto counts = count_labels(indices);
        VLabels filtered;
        for (size_t i = 0; i < counts.size(); ++i)
            if (counts[i] && counts[i] >= min_labels_discovered) filtered.push_back(this->label_encoder_.decode(i));
        return filtered;
    }

    // get_labels(indices, presence_ratio) for a batch of reads (the classify
    // loop over reads, annotated_dbg.cpp:88-110): one device call for all
    // reads when the matrix offers it (BRWTDevice, BinRelWTDevice), else one
    // get_labels per read
    std::vector<VLabels> get_labels_batch(const std::vector<std::vector<Index>> &reads,
                                          double presence_ratio) const {
        assert(presence_ratio >= 0 && presence_ratio <= 1);
        std::vector<Index> rows;
        std::vector<uint64_t> read_off{0}, lab_off;
        for (const auto &read : reads) {
            rows.insert(rows.end(), read.begin(), read.end());
            read_off.push_back(rows.size());
        }
        std::vector<uint32_t> codes;
        std::vector<VLabels> out(reads.size());
        if (!matrix_->labels_batch_csr(rows, read_off, presence_ratio, &lab_off, &codes)) {
            for (size_t r = 0; r < reads.size(); ++r) out[r] = get_labels(reads[r], presence_ratio);
            return out;
        }
        for (size_t r = 0; r < reads.size(); ++r)
            for (uint64_t i = lab_off[r]; i < lab_off[r + 1]; ++i)
                out[r].push_back(this->label_encoder_.decode(codes[i]));
        return out;
    }

    // get_top_labels for a batch of reads (classify --count-labels,
    // main.cpp:177): one device call when the matrix offers it, else one
    // get_top_labels per read
    std::vector<std::vector<std::pair<Label, size_t>>> get_top_labels_batch(
        const std::vector<std::vector<Index>> &reads, size_t num_top = static_cast<size_t>(-1)) const {
        std::vector<Index> rows;
        std::vector<uint64_t> read_off{0}, lab_off, counts;
        for (const auto &read : reads) {
            rows.insert(rows.end(), read.begin(), read.end());
            read_off.push_back(rows.size());
        }
        std::vector<uint32_t> codes;
        std::vector<std::vector<std::pair<Label, size_t>>> out(reads.size());
        if (!matrix_->top_labels_batch_csr(rows, read_off, num_top, &lab_off, &codes, &counts)) {
            for (size_t r = 0; r < reads.size(); ++r) out[r] = this->get_top_labels(reads[r], num_top);
            return out;
        }
        for (size_t r = 0; r < reads.size(); ++r)
            for (uint64_t i = lab_off[r]; i < lab_off[r + 1]; ++i)
                out[r].emplace_back(this->label_encoder_.decode(codes[i]), counts[i]);
        return out;
    }

    // annotate_static.cpp:96-109: the label encoder, then the matrix
    void serialize(const std::string &filename) const override {
        const std::string ext = AnnotatorExtension<BinaryMatrixType>::value();
        std::ofstream outstream(remove_suffix(filename, ext) + ext, std::ios::binary);
        if (!outstream.good()) throw std::ofstream::failure("Bad stream");
        this->label_encoder_.serialize(outstream);
        matrix_->serialize(outstream);
    }

    // annotate_static.cpp:111-130 (only the first file is loaded)
    bool merge_load(const std::vector<std::string> &filenames) override {
        if (filenames.size() > 1)
            std::cerr << "Warning: Can't merge static annotators."
                         " Only the first will be loaded."
                      << std::endl;
        const std::string ext = AnnotatorExtension<BinaryMatrixType>::value();
        std::ifstream instream(remove_suffix(filenames.at(0), ext) + ext, std::ios::binary);
        if (!instream.good()) return false;
        try {
            if (!matrix_) return false;
            return this->label_encoder_.load(instream) && matrix_->load(instream);
        } catch (...) {
            return false;
        }
    }

    uint64_t num_objects() const override { return matrix_->num_rows(); }
    size_t num_labels() const override { return this->label_encoder_.size(); }
    uint64_t num_relations() const override { return matrix_->num_relations(); }

    // the static representation has no dynamic actions (annotate_static.cpp:164-168)
    void set_labels(Index, const VLabels &) override { except_dyn(); }
    void add_label(Index, const Label &) override { except_dyn(); }
    void add_labels(Index, const VLabels &) override { except_dyn(); }
    void add_labels(const std::vector<Index> &, const VLabels &) override { except_dyn(); }
    void insert_rows(const std::vector<Index> &) override { except_dyn(); }

    const BinaryMatrixType &data() const { return *matrix_; }

    // annotate_static.cpp:149-162, batched
    std::vector<uint64_t> count_labels(const std::vector<Index> &indices) const override {
        std::vector<uint64_t> counter(num_labels(), 0);
        if (indices.empty()) return counter;
        for (const auto &row : matrix_->get_rows(indices))
            for (auto col : row) counter[col]++;
        return counter;
    }

  private:
    static std::shared_ptr<BinaryMatrixType> make_default() {
        if constexpr (std::is_default_constructible<BinaryMatrixType>::value && !std::is_abstract<BinaryMatrixType>::value)
            return std::make_shared<BinaryMatrixType>();
        else
            return nullptr;
    }
    void except_dyn() const { throw std::runtime_error("Dynamic actions are not supported in static representation"); }

    std::shared_ptr<BinaryMatrixType> matrix_;
};

}  // namespace mbrwt_host

// hdfs_ec.hpp -- header-only C++ mirror of hdfs-native's erasure-coding host
// interface, layered on the C ABI (include/hdfs_ec_amd.h).  The reference is
// Rust (no Rust toolchain in this image), so this is the host side a C++
// consumer links; the Rust-side binding is shown in INTEGRATION.md.
//
// Mirrors (hdfs-native 0.14.1):
//   Coder::{new, gen_rs_matrix, encode, decode}   rust/src/ec/gf256.rs:25-138
//   EcSchema + geometry helpers + ec_decode        rust/src/ec/mod.rs:14-89
//   resolve_ec_policy                              rust/src/ec/mod.rs:93-144
//   CellBuffer::{write, is_full, is_empty, encode} rust/src/hdfs/block_writer.rs:771-852
// Errors: the reference's Result<_, HdfsError> becomes a thrown HdfsError
// with the same kind; its assert!/panic paths throw std::invalid_argument.
#pragma once

#include <cstdint>
#include <cstring>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/hdfs_ec_amd.h"

namespace hdfs_native {

enum class HdfsErrorKind { ErasureCodingError, UnsupportedErasureCodingPolicy, Device };

// rust/src/error.rs:32-35 (+ a device kind for HIP failures)
class HdfsError : public std::runtime_error {
   public:
    HdfsError(HdfsErrorKind k, const std::string& msg) : std::runtime_error(msg), kind(k) {}
    HdfsErrorKind kind;
};

namespace ec {

using Bytes = std::vector<uint8_t>;

inline void check(int rc) {
    switch (rc) {
        case HEC_OK: return;
        case HEC_ERR_NOT_ENOUGH_SHARDS:
            throw HdfsError(HdfsErrorKind::ErasureCodingError, "erasure coding error: Not enough valid shards");
        case HEC_ERR_UNSUPPORTED_CODEC:
            throw HdfsError(HdfsErrorKind::UnsupportedErasureCodingPolicy, hec_strerror(rc));
        case HEC_ERR_INVALID_ARG:
        case HEC_ERR_SINGULAR: throw std::invalid_argument(hec_strerror(rc));
        default: throw HdfsError(HdfsErrorKind::Device, std::string(hec_strerror(rc)) + ": " + hec_last_error());
    }
}

// gf256.rs:25-138 on one MI355X.
class Coder {
   public:
    Coder(size_t data_units, size_t parity_units, int device = 0) : k_(data_units), m_(parity_units) {
        hec_coder_t* h = nullptr;
        check(hec_coder_create(data_units, parity_units, device, &h));
        h_.reset(h);
    }

    size_t data_units() const { return k_; }
    size_t parity_units() const { return m_; }
    hec_coder_t* handle() const { return h_.get(); }

    // gf256.rs:40-57
    static std::vector<std::vector<uint8_t>> gen_rs_matrix(size_t data_units, size_t parity_units) {
        std::vector<uint8_t> flat((data_units + parity_units) * data_units);
        check(hec_gen_rs_matrix(data_units, parity_units, flat.data()));
        std::vector<std::vector<uint8_t>> rows(data_units + parity_units);
        for (size_t r = 0; r < rows.size(); r++)
            rows[r].assign(flat.begin() + r * data_units, flat.begin() + (r + 1) * data_units);
        return rows;
    }

    // gf256.rs:61-80: asserts data.len() == k and equal lengths
    std::vector<Bytes> encode(const std::vector<Bytes>& data) const {
        if (data.size() != k_) throw std::invalid_argument("encode: data.len() != data_units");
        const size_t n = data[0].size();
        for (const Bytes& d : data)
            if (d.size() != n) throw std::invalid_argument("encode: shards of unequal length");
        std::vector<Bytes> parity(m_, Bytes(n));
        std::vector<const uint8_t*> in(k_);
        std::vector<uint8_t*> out(m_);
        for (size_t i = 0; i < k_; i++) in[i] = data[i].data();
        for (size_t j = 0; j < m_; j++) out[j] = parity[j].data();
        check(hec_encode(h_.get(), in.data(), n, out.data()));
        return parity;
    }

    // gf256.rs:84-137: fills missing data slots in place; parity stays None
    void decode(std::vector<std::optional<Bytes>>& data) const {
        if (data.size() != k_ + m_) throw std::invalid_argument("decode: need data_units + parity_units slots");
        size_t n = 0;
        bool any = false, data_missing = false;
        for (size_t i = 0; i < data.size(); i++) {
            if (data[i]) {
                n = data[i]->size();
                any = true;
            } else if (i < k_) {
                data_missing = true;
            }
        }
        if (!data_missing) return;  // gf256.rs:102-105
        if (!any) check(HEC_ERR_NOT_ENOUGH_SHARDS);
        std::vector<const uint8_t*> in(k_ + m_, nullptr);
        std::vector<Bytes> rec(k_);
        std::vector<uint8_t*> out(k_ + m_, nullptr);
        for (size_t i = 0; i < data.size(); i++)
            if (data[i]) in[i] = data[i]->data();
        for (size_t i = 0; i < k_; i++)
            if (!data[i]) {
                rec[i].resize(n);
                out[i] = rec[i].data();
            }
        check(hec_decode(h_.get(), in.data(), n, out.data()));
        for (size_t i = 0; i < k_; i++)
            if (!data[i]) data[i] = std::move(rec[i]);
    }

   private:
    struct Deleter {
        void operator()(hec_coder_t* c) const { hec_coder_destroy(c); }
    };
    size_t k_, m_;
    std::unique_ptr<hec_coder_t, Deleter> h_;
};

constexpr const char* kRsCodec = "rs";
constexpr const char* kRsLegacyCodec = "rs-legacy";
constexpr const char* kXorCodec = "xor";
constexpr size_t kDefaultCellSize = 1024 * 1024;  // mod.rs:12

// mod.rs:14-89
struct EcSchema {
    std::string codec_name;
    size_t data_units = 0;
    size_t parity_units = 0;
    size_t cell_size = 0;

    size_t row_size() const { return cell_size * data_units; }
    size_t cell_for_offset(size_t offset) const { return offset / cell_size; }
    size_t row_for_cell(size_t cell_id) const { return cell_id / data_units; }
    size_t offset_for_row(size_t row_id) const { return row_id * cell_size; }

    // mod.rs:40-60: bytes of block `index` in a block group of block_size bytes
    size_t max_offset(size_t index, size_t block_size) const {
        if (index >= data_units) index = 0;  // parity cells are as long as block 0
        const size_t full_rows = block_size / row_size();
        const size_t full_row_bytes = full_rows * row_size();
        const size_t remaining = block_size - full_row_bytes;
        size_t last;
        if (remaining < index * cell_size)
            last = 0;
        else if (remaining > (index + 1) * cell_size)
            last = cell_size;
        else
            last = remaining - index * cell_size;
        return full_rows * cell_size + last;
    }

    // mod.rs:62-89: decode (only codec "rs") when a data shard is missing,
    // then cut every data shard into cell_size cells, row by row.
    std::vector<Bytes> ec_decode(std::vector<std::optional<Bytes>> vertical, const Coder* coder = nullptr) const {
        bool all_data = true;
        for (size_t i = 0; i < data_units && i < vertical.size(); i++) all_data &= bool(vertical[i]);
        if (!all_data) {
            if (codec_name != kRsCodec)
                throw HdfsError(HdfsErrorKind::UnsupportedErasureCodingPolicy, "codec: " + codec_name);
            if (coder) {
                coder->decode(vertical);
            } else {
                Coder c(data_units, parity_units);  // mod.rs:71 builds a Coder per call
                c.decode(vertical);
            }
        }
        // mod.rs:82-86: Bytes::split_to(cell_size) panics when fewer bytes are
        // left (the reader pads every cell to cell_size, block_reader.rs:
        // 370-371, so that is a programming error): throw std::out_of_range,
        // never clamp
        std::vector<Bytes> cells;
        std::vector<size_t> off(data_units, 0);
        while (vertical[0] && off[0] < vertical[0]->size()) {
            for (size_t i = 0; i < data_units; i++) {
                const Bytes& v = *vertical[i];
                if (off[i] + cell_size > v.size())
                    throw std::out_of_range("split_to out of bounds: shard " + std::to_string(i) + " has " +
                                            std::to_string(v.size() - std::min(off[i], v.size())) +
                                            " bytes left, cell_size " + std::to_string(cell_size));
                cells.emplace_back(v.begin() + off[i], v.begin() + off[i] + cell_size);
                off[i] += cell_size;
            }
        }
        return cells;
    }
};

// hdfs::ErasureCodingPolicyProto, the fields resolve_ec_policy reads
struct ErasureCodingPolicy {
    uint32_t id = 0;
    struct Schema {
        std::string codec_name;
        uint32_t data_units = 0, parity_units = 0;
    };
    std::optional<Schema> schema;
    uint32_t cell_size = 0;
};

// mod.rs:93-144
inline EcSchema resolve_ec_policy(const ErasureCodingPolicy& p) {
    if (p.schema) return {p.schema->codec_name, p.schema->data_units, p.schema->parity_units, p.cell_size};
    switch (p.id) {
        case 1: return {kRsCodec, 6, 3, kDefaultCellSize};        // RS-6-3-1024k
        case 2: return {kRsCodec, 3, 2, kDefaultCellSize};        // RS-3-2-1024k
        case 3: return {kRsLegacyCodec, 6, 3, kDefaultCellSize};  // RS-LEGACY-6-3-1024k
        case 4: return {kXorCodec, 2, 1, kDefaultCellSize};       // XOR-2-1-1024k
        case 5: return {kRsCodec, 10, 4, kDefaultCellSize};       // RS-10-4-1024k
        default:
            throw HdfsError(HdfsErrorKind::UnsupportedErasureCodingPolicy, "ID: " + std::to_string(p.id));
    }
}

// block_writer.rs:771-852: stripes user bytes into k cell buffers; encode()
// zero-pads all buffers to buffers[0].len(), encodes, returns the k data
// cells at their original lengths followed by the m parity cells.
class CellBuffer {
   public:
    explicit CellBuffer(const EcSchema& s, int device = 0)
        : buffers_(s.data_units), cell_size_(s.cell_size), coder_(s.data_units, s.parity_units, device) {
        for (Bytes& b : buffers_) b.reserve(cell_size_);
    }

    // block_writer.rs:791-805: consumes from `buf` until the row is full
    void write(Bytes& buf, size_t& consumed) {
        while (consumed < buf.size() && current_ < buffers_.size()) {
            Bytes& cur = buffers_[current_];
            const size_t take = std::min(cell_size_ - cur.size(), buf.size() - consumed);
            cur.insert(cur.end(), buf.begin() + consumed, buf.begin() + consumed + take);
            consumed += take;
            if (cur.size() == cell_size_) current_++;
        }
    }

    bool is_full() const { return current_ == buffers_.size(); }
    bool is_empty() const { return buffers_[0].empty(); }

    std::vector<Bytes> encode() {
        const size_t slice = buffers_[0].size();
        std::vector<Bytes> out;
        out.reserve(buffers_.size() + coder_.parity_units());
        std::vector<Bytes> padded(buffers_.size());
        for (size_t i = 0; i < buffers_.size(); i++) {
            padded[i] = buffers_[i];
            padded[i].resize(slice, 0);
        }
        std::vector<Bytes> parity = coder_.encode(padded);
        for (Bytes& b : buffers_) {
            out.push_back(std::move(b));
            b = Bytes();
            b.reserve(cell_size_);
        }
        current_ = 0;
        for (Bytes& p : parity) out.push_back(std::move(p));
        return out;
    }

   private:
    std::vector<Bytes> buffers_;
    size_t cell_size_;
    size_t current_ = 0;
    Coder coder_;
};

}  // namespace ec
}  // namespace hdfs_native

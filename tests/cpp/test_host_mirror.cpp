// test_host_mirror.cpp -- exercises the C++ host mirror (hdfs_ec.hpp) the way
// the reference's own tests exercise its EC path.
//   ./test_host_mirror cpu   -> prints JSON lines (policy resolution,
//                               max_offset grid) that tests/test_host_mirror.py
//                               compares with the oracle
//   ./test_host_mirror gpu   -> end-to-end striped write + faulty read on the
//                               GPU, restating rust/tests/test_ec.rs:88-158
//                               (counter files, 0..m-1 failed shards must read
//                               back exactly, m+1 failures must error)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../hdfs-native_amd/csrc/hdfs_ec.hpp"

using namespace hdfs_native;
using namespace hdfs_native::ec;

static int cpu_mode() {
    for (uint32_t id = 1; id <= 6; id++) {
        ErasureCodingPolicy p;
        p.id = id;
        try {
            EcSchema s = resolve_ec_policy(p);
            std::printf("{\"policy\": %u, \"codec\": \"%s\", \"k\": %zu, \"m\": %zu, \"cell\": %zu}\n", id,
                        s.codec_name.c_str(), s.data_units, s.parity_units, s.cell_size);
        } catch (const HdfsError& e) {
            std::printf("{\"policy\": %u, \"error\": \"%s\"}\n", id, e.what());
        }
    }
    ErasureCodingPolicy custom;
    custom.id = 99;
    custom.schema = ErasureCodingPolicy::Schema{"rs", 4, 2};
    custom.cell_size = 65536;
    EcSchema cs = resolve_ec_policy(custom);
    std::printf("{\"policy\": 99, \"codec\": \"%s\", \"k\": %zu, \"m\": %zu, \"cell\": %zu}\n", cs.codec_name.c_str(),
                cs.data_units, cs.parity_units, cs.cell_size);
    EcSchema s{"rs", 3, 2, 16};
    for (size_t index = 0; index < 5; index++)
        for (size_t bs = 0; bs <= 200; bs += 7)
            std::printf("{\"max_offset\": [%zu, %zu, %zu]}\n", index, bs, s.max_offset(index, bs));
    auto m = Coder::gen_rs_matrix(6, 3);
    std::printf("{\"rs63_row6\": [%d, %d, %d, %d, %d, %d]}\n", m[6][0], m[6][1], m[6][2], m[6][3], m[6][4], m[6][5]);
    // ec_decode's cell split (mod.rs:82-86) with every data shard present (no
    // decode, no device): whole cells split row by row; a shard shorter than
    // the next cell is Bytes::split_to's panic -> std::out_of_range
    EcSchema sp{"rs", 3, 2, 16};
    std::vector<std::optional<Bytes>> v = {Bytes(32, 1), Bytes(32, 2), Bytes(32, 3), std::nullopt, std::nullopt};
    const std::vector<Bytes> cells = sp.ec_decode(v);
    std::printf("{\"split_cells\": [%zu, %d, %d]}\n", cells.size(), cells.empty() ? -1 : int(cells[1][0]),
                cells.size() < 4 ? -1 : int(cells[3][0]));
    v[2] = Bytes(20, 3);
    try {
        sp.ec_decode(v);
        std::printf("{\"split_short\": \"no error\"}\n");
    } catch (const std::out_of_range&) {
        std::printf("{\"split_short\": \"out_of_range\"}\n");
    }
    return 0;
}

// ---- GPU: striped write through CellBuffer, faulty striped read ----------

static Bytes counter_file(size_t bytes) {
    Bytes f(bytes);
    for (size_t i = 0; i + 4 <= bytes; i += 4) {
        uint32_t v = uint32_t(i / 4);
        f[i] = uint8_t(v >> 24);
        f[i + 1] = uint8_t(v >> 16);
        f[i + 2] = uint8_t(v >> 8);
        f[i + 3] = uint8_t(v);
    }
    return f;
}

// StripedBlockWriter::write + close (block_writer.rs:904-1035) for a single
// block group: every full row and the final partial row go through
// CellBuffer::encode; shard i accumulates its cells.
static std::vector<Bytes> write_block_group(const EcSchema& s, const Bytes& file) {
    CellBuffer cb(s);
    std::vector<Bytes> shards(s.data_units + s.parity_units);
    Bytes buf = file;
    size_t consumed = 0;
    auto flush = [&] {
        std::vector<Bytes> cells = cb.encode();
        for (size_t i = 0; i < cells.size(); i++) shards[i].insert(shards[i].end(), cells[i].begin(), cells[i].end());
    };
    while (consumed < buf.size()) {
        cb.write(buf, consumed);
        if (cb.is_full()) flush();
    }
    if (!cb.is_empty()) flush();
    return shards;
}

// StripedBlockStream::read_slice (block_reader.rs:480-554) with the first
// `faults` shards failed: per row, read one cell per shard from the first k
// healthy shards (CellReader pads short cells with zeros, :343-378), decode,
// concatenate, trim to the file length.
static Bytes read_block_group(const EcSchema& s, const std::vector<Bytes>& shards, size_t file_len, size_t faults,
                              const Coder& coder) {
    Bytes out;
    const size_t rows = (file_len + s.row_size() - 1) / s.row_size();
    for (size_t row = 0; row < rows; row++) {
        std::vector<std::optional<Bytes>> slice(s.data_units + s.parity_units);
        size_t good = 0;
        for (size_t i = 0; i < slice.size() && good < s.data_units; i++) {
            if (i < faults) continue;
            Bytes cell(s.cell_size, 0);
            const size_t off = row * s.cell_size;
            if (off < shards[i].size()) {
                const size_t n = std::min(s.cell_size, shards[i].size() - off);
                std::memcpy(cell.data(), shards[i].data() + off, n);
            }
            slice[i] = std::move(cell);
            good++;
        }
        std::vector<Bytes> cells = s.ec_decode(std::move(slice), &coder);
        for (const Bytes& c : cells) out.insert(out.end(), c.begin(), c.end());
    }
    out.resize(file_len);
    return out;
}

// Writes the shards of one striped write to $HEC_MIRROR_DUMP/<k>_<m>_<size>_<i>.bin
// so the Python test can pin their bytes against the oracle.
static void dump_shards(const EcSchema& s, size_t size, const std::vector<Bytes>& shards) {
    const char* dir = std::getenv("HEC_MIRROR_DUMP");
    if (!dir) return;
    for (size_t i = 0; i < shards.size(); i++) {
        const std::string path = std::string(dir) + "/" + std::to_string(s.data_units) + "_" +
                                 std::to_string(s.parity_units) + "_" + std::to_string(size) + "_" +
                                 std::to_string(i) + ".bin";
        FILE* f = std::fopen(path.c_str(), "wb");
        if (!f) continue;
        if (!shards[i].empty()) std::fwrite(shards[i].data(), 1, shards[i].size(), f);
        std::fclose(f);
    }
}

static int gpu_mode() {
    int failures = 0;
    const size_t cell = 65536;
    for (auto [k, m] : {std::pair<size_t, size_t>{3, 2}, {6, 3}, {10, 4}}) {
        EcSchema s{"rs", k, m, cell};
        Coder coder(k, m);
        // rust/tests/test_ec.rs:77-87
        const size_t sizes[] = {16, cell, cell - 4, cell + 4, cell * k * 5, cell * k * 5 - 4, cell * k * 5 + 4};
        for (size_t size : sizes) {
            const Bytes file = counter_file(size);
            const std::vector<Bytes> shards = write_block_group(s, file);
            if (size == cell * k * 5 + 4 || size == cell - 4) dump_shards(s, size, shards);
            for (size_t faults = 0; faults < m; faults++) {
                const Bytes back = read_block_group(s, shards, size, faults, coder);
                if (back != file) {
                    std::printf("FAIL rs(%zu,%zu) size=%zu faults=%zu\n", k, m, size, faults);
                    failures++;
                }
            }
            // m+1 failures: not enough shards -> ErasureCodingError
            bool threw = false;
            try {
                read_block_group(s, shards, size, m + 1, coder);
            } catch (const HdfsError& e) {
                threw = e.kind == HdfsErrorKind::ErasureCodingError;
            }
            if (!threw) {
                std::printf("FAIL rs(%zu,%zu) size=%zu: %zu failures did not error\n", k, m, size, m + 1);
                failures++;
            }
        }
        std::printf("rs(%zu,%zu) striped write/read round trips done\n", k, m);
    }
    // Concurrent callers (the reference's Coder is Send + Sync, called from
    // many tokio workers at once): 8 native threads share one Coder through
    // striped writes and faulty reads of different files.
    {
        const size_t k = 6, m = 3;
        EcSchema s{"rs", k, m, cell};
        Coder shared(k, m);
        std::vector<int> bad(8, 0);
        std::vector<std::thread> th;
        for (int t = 0; t < 8; t++)
            th.emplace_back([&, t] {
                try {
                    for (int it = 0; it < 3; it++) {
                        const size_t size = cell * k * size_t(1 + (t + it) % 3) + size_t(4 * t);
                        const Bytes file = counter_file(size);
                        const std::vector<Bytes> shards = write_block_group(s, file);
                        const Bytes back = read_block_group(s, shards, size, size_t((t + it) % m + 1), shared);
                        if (back != file) bad[t]++;
                    }
                } catch (...) {
                    bad[t]++;
                }
            });
        for (auto& x : th) x.join();
        for (int t = 0; t < 8; t++)
            if (bad[t]) {
                std::printf("FAIL concurrent thread %d\n", t);
                failures++;
            }
        std::printf("8 threads on one shared coder done\n");
    }
    // unsupported codec on the read path (mod.rs:74-78)
    try {
        EcSchema x{"xor", 2, 1, 16};
        std::vector<std::optional<Bytes>> v = {std::nullopt, Bytes(16, 1), Bytes(16, 1)};
        x.ec_decode(v);
        std::printf("FAIL xor codec decoded\n");
        failures++;
    } catch (const HdfsError& e) {
        if (e.kind != HdfsErrorKind::UnsupportedErasureCodingPolicy) failures++;
    }
    std::printf(failures ? "FAILED %d\n" : "ALL OK\n", failures);
    return failures ? 1 : 0;
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "cpu";
    try {
        return mode == "gpu" ? gpu_mode() : cpu_mode();
    } catch (const std::exception& e) {
        std::printf("EXCEPTION %s\n", e.what());
        return 2;
    }
}

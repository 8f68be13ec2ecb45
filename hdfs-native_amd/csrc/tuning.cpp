// tuning.cpp -- the CU-count cache and, in the HEC_EXPERIMENTAL measurement
// build only, hec_tune_set's knobs as atomics (see tuning.hpp).
#include "tuning.hpp"

#include <hip/hip_runtime.h>

#include <atomic>

#include "../../include/hdfs_ec_amd.h"

namespace hec {

namespace {

std::atomic<int> g_cus[64];

#ifdef HEC_EXPERIMENTAL
constexpr int kKeys = 33;
std::atomic<int> g_knob[kKeys + 1];  // index = key; zero-initialised (static storage)
std::atomic<int> g_nt{-1};           // key 2 defaults to -1 (non-temporal on)

int load(int key) { return g_knob[key].load(std::memory_order_relaxed); }
#endif

}  // namespace

#ifdef HEC_EXPERIMENTAL
Tune tune_snapshot() {
    Tune t;
    t.unroll = load(1);
    t.nt = g_nt.load(std::memory_order_relaxed);
    t.blocks_per_cu = load(3);
    t.block = load(4);
    t.pipeline = load(5);
    t.drain = load(6);
    t.grid = load(7);
    t.group = load(8);
    t.crc_unfused = load(9);
    t.fused_slabs = load(10);
    t.crc_variant = load(11);
    t.crc_prefetch = load(12);
    t.store_pol = load(13);
    t.host_copy_threads = load(14);
    t.burst_tiles = load(15);
    t.fused_wpe = load(16);
    t.call_piece_kib = load(17);
    t.unaligned = load(18);
    t.fused_pair = load(19);
    t.mixed_skip = load(20);
    t.fused_split = load(21);
    t.fused_bsl = load(22);
    t.matmul_bsl = load(23);
    t.jit_pfd = load(24);
    t.col_rot = load(25);
    t.mixed_wq = load(26);
    t.matmul_wq = load(27);
    t.fused_wq = load(28);
    t.crc_wq = load(29);
    t.crc_sums_nt = load(30);
    t.crc_runs = load(31);
    t.matmul_pair = load(32);
    t.crc_block = load(33);
    return t;
}

int tune_store(int key, int value) {
    bool ok = false;
    switch (key) {
        case 1: ok = value == 0 || value == 1 || value == 2 || value == 3 || value == 4 || value == 8; break;
        case 2:
            g_nt.store(value < 0 ? -1 : (value ? 1 : 0), std::memory_order_relaxed);
            return HEC_OK;
        case 3: ok = value >= 0 && value <= 16; break;
        case 4: ok = value == 0 || value == 256 || value == 512; break;
        case 5: ok = value >= 0 && value <= 2; break;
        case 6: ok = value >= 0 && value <= 2; break;
        case 7: ok = value >= 0 && value <= 65536; break;
        case 8: ok = value >= 0 && value <= 65536; break;
        case 9: value = value ? 1 : 0; ok = true; break;
        case 10: ok = value == 0 || value == 4 || value == 8; break;
        case 11: ok = value == 0 || value == 1 || value == 2 || value == 3 || value == 4 || value == 5 || value == 6 ||
                      value == 7 || value == 9 || value == 10 || value == 11 || value == 12;  // 13 retired
            break;
        case 12: ok = value >= 0 && value <= 2; break;
        case 13: ok = value == 0; break;  // retired
        case 14: ok = value >= 0 && value <= 64; break;
        case 15: ok = value == 0; break;  // retired
        case 16: ok = value == 0 || value == 2 || value == 3; break;
        case 17: ok = value >= 0 && value <= 65536 && (value & 3) == 0; break;
        case 18: ok = value == 0 || value == 1; break;
        case 19: ok = value >= 0 && value <= 2; break;
        case 20: ok = value >= 0 && value <= 2; break;
        case 21: ok = value == 0 || value == 1; break;  // 2 / 3 (role split) retired
        case 22: ok = value == 0 || value == 1; break;
        case 23: ok = value == 0 || value == 1; break;
        case 24: ok = value >= 0 && value <= 5; break;
        case 25: ok = value >= 0 && value <= 4096; break;
        case 26: ok = value >= 0 && value <= 4; break;
        case 27: ok = value >= 0 && value <= 3; break;
        case 28: ok = value >= 0 && value <= 2; break;
        case 29: ok = value == 0 || value == 1 || value == 2 || value == 4 || value == 8 || value == 16; break;
        case 30: ok = value == 0 || value == 1; break;
        case 31: ok = value == 0 || value == 2 || value == 4 || value == 8 || value == 16; break;
        case 32: ok = value == 0 || value == 1; break;
        case 33: ok = value == 0 || value == 768; break;
        default: ok = false;
    }
    if (!ok) return HEC_ERR_INVALID_ARG;
    g_knob[key].store(value, std::memory_order_relaxed);
    return HEC_OK;
}
#endif

int num_cus(int dev) {
    if (dev < 0 || dev >= 64) return 256;
    int v = g_cus[dev].load(std::memory_order_relaxed);
    if (v > 0) return v;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    g_cus[dev].store(v, std::memory_order_relaxed);  // every racing writer stores the same value
    return v;
}

}  // namespace hec

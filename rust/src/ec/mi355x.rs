//! MI355X erasure-coding engine behind hdfs-native's internal EC functions.
//!
//! FFI to the C ABI in `include/hdfs_ec_amd.h` (library
//! `hdfs-native_amd/lib/libhdfs_ec_amd.so`), compiled only with the `mi355x`
//! cargo feature (see `rust/Cargo.toml.mi355x` and `rust/build_mi355x.rs`).
//! This file is written for hdfs-native 0.14.1's `rust/src/ec/` and is NOT
//! compiled in this repository's image (no cargo/rustc); `tests/cpp/
//! shim_replay.c` replays its exact C call sequence against the engine.
//!
//! It replaces, with the same contracts:
//!   * `Coder::new`     (`rust/src/ec/gf256.rs:32-38`)
//!   * `Coder::encode`  (`gf256.rs:61-80`): panics on a wrong shard count or
//!     unequal / zero lengths, like the reference's asserts (`gf256.rs:62-65`,
//!     `matrix.rs:57`); otherwise infallible;
//!   * `Coder::decode`  (`gf256.rs:84-137`): fills only missing DATA slots,
//!     first-k-present survivors, `Err(ErasureCodingError("Not enough valid
//!     shards"))` when fewer than k are present; parity slots are never
//!     touched.
//! and adds the batched forms the striped writer/reader can use instead of
//! one call per 1 MiB row.  `PooledCoder` is what `Coder::new` holds when the
//! `mi355x` feature forwards the reference's `Coder` (rust/patches/
//! ec_mi355x.patch): the reference builds a Coder per decoded row
//! (`ec/mod.rs:71`), so it takes an idle engine coder from the process-wide
//! pool (`hec_coder_acquire`) and gives it back on drop.  `Coder::new` stays
//! infallible: without a GPU the pool hands out an engine host-only coder,
//! and if even that fails the patched `Coder` keeps `None` and runs the
//! reference CPU path.  The striped writer and reader keep calling one row
//! at a time on pageable cells, which the engine codes with its host routine
//! (DESIGN.md §1 measures the device route at those call shapes: it loses).
//! `GpuCoder::encode_rows` / `decode_rows` are the pinned-memory batched
//! forms for callers that hold many rows at once (a reconstruct worker);
//! `GpuCoder::encode_device` / `decode_device` with `DeviceBuffer` the
//! device-resident forms (the patch's `mi355x` group of rust/benches/ec.rs).

use std::ffi::{c_char, c_int, c_void, CStr};

use bytes::{Bytes, BytesMut};

use crate::{HdfsError, Result};

#[repr(C)]
pub struct HecCoder {
    _private: [u8; 0],
}

#[repr(C)]
pub struct HecGroup {
    _private: [u8; 0],
}

const HEC_OK: c_int = 0;
const HEC_ERR_INVALID_ARG: c_int = -1;
const HEC_ERR_NOT_ENOUGH_SHARDS: c_int = -2;
const HEC_ERR_UNSUPPORTED_CODEC: c_int = -3;
const HEC_ERR_CHECKSUM: c_int = -7;
/// `device` of an engine host-only coder (include/hdfs_ec_amd.h).
const HEC_DEVICE_HOST: c_int = -2;

unsafe extern "C" {
    fn hec_abi_version() -> c_int;
    fn hec_strerror(rc: c_int) -> *const c_char;
    fn hec_last_error() -> *const c_char;
    fn hec_coder_create_codec(codec: *const c_char, k: usize, m: usize, device: c_int,
                              out: *mut *mut HecCoder) -> c_int;
    fn hec_coder_destroy(c: *mut HecCoder);
    fn hec_coder_acquire(codec: *const c_char, k: usize, m: usize, device: c_int, out: *mut *mut HecCoder) -> c_int;
    fn hec_coder_release(c: *mut HecCoder);
    fn hec_coder_device(c: *const HecCoder) -> c_int;
    fn hec_encode_rows_host(c: *mut HecCoder, h_data: *const u8, data_len: usize, h_parity: *mut u8,
                            cell_len: usize, chunk_stripes: usize) -> c_int;
    fn hec_decode_rows_host(c: *mut HecCoder, h_vertical: *const *const u8, vertical_len: *const usize,
                            cell_len: usize, h_file: *mut u8, file_len: usize, chunk_rows: usize) -> c_int;
    fn hec_encode(c: *mut HecCoder, data: *const *const u8, n: usize, parity: *const *mut u8) -> c_int;
    fn hec_decode(c: *mut HecCoder, shards: *const *const u8, n: usize, out: *const *mut u8) -> c_int;
    fn hec_encode_host_batch(c: *mut HecCoder, h_data: *const u8, h_parity: *mut u8, cell_len: usize,
                             stripes: usize, chunk_stripes: usize) -> c_int;
    fn hec_decode_host_batch(c: *mut HecCoder, h_vertical: *const *const u8, cell_len: usize, rows: usize,
                             h_file: *mut u8, chunk_rows: usize) -> c_int;
    fn hec_decode_verify_device(c: *mut HecCoder, checksum_type: c_int, d_shards: *const *const u8,
                                shard_strides: *const usize, d_out: *const *mut u8, out_strides: *const usize,
                                cell_len: usize, stripes: usize, bytes_per_checksum: usize, d_sums: *const u8,
                                d_bad: *mut u8, stream: *mut c_void) -> c_int;
    fn hec_encode_device(c: *mut HecCoder, d_data: *const *const u8, data_strides: *const usize,
                         d_parity: *const *mut u8, parity_strides: *const usize, cell_len: usize, stripes: usize,
                         stream: *mut c_void) -> c_int;
    fn hec_decode_device(c: *mut HecCoder, d_shards: *const *const u8, shard_strides: *const usize,
                         d_out: *const *mut u8, out_strides: *const usize, cell_len: usize, stripes: usize,
                         stream: *mut c_void) -> c_int;
    fn hec_device_alloc(device: c_int, bytes: usize, flags: u32, out: *mut *mut c_void) -> c_int;
    fn hec_device_free(device: c_int, ptr: *mut c_void) -> c_int;
    fn hec_device_copy(device: c_int, dst: *mut c_void, src: *const c_void, bytes: usize) -> c_int;
    fn hec_device_synchronize(device: c_int, stream: *mut c_void) -> c_int;
    fn hec_group_create(codec: *const c_char, k: usize, m: usize, devices: *const c_int, n_devices: usize,
                        out: *mut *mut HecGroup) -> c_int;
    fn hec_group_destroy(g: *mut HecGroup);
    fn hec_group_encode_host_batch(g: *mut HecGroup, h_data: *const u8, h_parity: *mut u8, cell_len: usize,
                                   stripes: usize, chunk_stripes: usize) -> c_int;
    fn hec_group_decode_host_batch(g: *mut HecGroup, h_vertical: *const *const u8, cell_len: usize,
                                   rows: usize, h_file: *mut u8, chunk_rows: usize) -> c_int;
}

/// The ABI revision this shim is written against (include/hdfs_ec_amd.h).
const ABI_VERSION: c_int = 5;

/// Status -> the reference's error kinds (rust/src/error.rs:32-39).
fn err(rc: c_int) -> HdfsError {
    match rc {
        HEC_ERR_NOT_ENOUGH_SHARDS => HdfsError::ErasureCodingError("Not enough valid shards".to_string()),
        HEC_ERR_UNSUPPORTED_CODEC => HdfsError::UnsupportedErasureCodingPolicy("engine codec".to_string()),
        HEC_ERR_CHECKSUM => HdfsError::ChecksumError,
        HEC_ERR_INVALID_ARG => HdfsError::InvalidArgument(status_text(rc)),
        _ => HdfsError::InternalError(format!("{}: {}", status_text(rc), last_error())),
    }
}

fn status_text(rc: c_int) -> String {
    unsafe { CStr::from_ptr(hec_strerror(rc)).to_string_lossy().into_owned() }
}

fn last_error() -> String {
    unsafe { CStr::from_ptr(hec_last_error()).to_string_lossy().into_owned() }
}

fn check(rc: c_int) -> Result<()> {
    if rc == HEC_OK { Ok(()) } else { Err(err(rc)) }
}

/// A coder bound to one MI355X (`hec_coder_t`).  The C ABI serialises the
/// host-buffer calls of one coder internally, so it may be shared.
pub struct GpuCoder {
    raw: *mut HecCoder,
    data_units: usize,
    parity_units: usize,
    device: i32,
}

unsafe impl Send for GpuCoder {}
unsafe impl Sync for GpuCoder {}

impl GpuCoder {
    /// `Coder::new` on device `device` for codec "rs" (or "xor", "rs-legacy").
    pub fn new(codec: &str, data_units: usize, parity_units: usize, device: i32) -> Result<Self> {
        assert_eq!(unsafe { hec_abi_version() }, ABI_VERSION, "libhdfs_ec_amd ABI mismatch");
        let name = std::ffi::CString::new(codec).map_err(|_| HdfsError::InvalidArgument(codec.to_string()))?;
        let mut raw = std::ptr::null_mut();
        check(unsafe { hec_coder_create_codec(name.as_ptr(), data_units, parity_units, device, &mut raw) })?;
        Ok(Self { raw, data_units, parity_units, device })
    }

    /// The coder's device ordinal.
    pub fn device(&self) -> i32 {
        self.device
    }

    /// Batched `Coder::encode` on stripes already in HBM (`hec_encode_device`):
    /// shard i of stripe s at `data[i] + s * data_strides[i]`, parity row j at
    /// `parity[j] + s * parity_strides[j]`; enqueued on `stream` (null = the
    /// device's default stream), complete after `synchronize`.
    ///
    /// # Safety
    /// Device pointers valid for `stripes` cells of `cell` bytes in that
    /// layout, on this coder's device; `stream` belongs to it.
    #[allow(clippy::too_many_arguments)]
    pub unsafe fn encode_device(&self, data: &[*const u8], data_strides: &[usize], parity: &[*mut u8],
                                parity_strides: &[usize], cell: usize, stripes: usize,
                                stream: *mut c_void) -> Result<()> {
        let (k, m) = (self.data_units, self.parity_units);
        assert!(data.len() == k && data_strides.len() == k, "one slot per data shard");
        assert!(parity.len() == m && parity_strides.len() == m, "one slot per parity shard");
        check(unsafe {
            hec_encode_device(self.raw, data.as_ptr(), data_strides.as_ptr(), parity.as_ptr(),
                              parity_strides.as_ptr(), cell, stripes, stream)
        })
    }

    /// Batched `Coder::decode` on stripes already in HBM (`hec_decode_device`),
    /// one erasure pattern for the batch: `shards[k+m]` (null = missing),
    /// missing data shard i rebuilt into `out[i]` (the other `out` slots are
    /// never written; null is fine there).  `Err(ErasureCodingError)` when
    /// fewer than k shards are present.
    ///
    /// # Safety
    /// As `encode_device`.
    #[allow(clippy::too_many_arguments)]
    pub unsafe fn decode_device(&self, shards: &[*const u8], shard_strides: &[usize], out: &[*mut u8],
                                out_strides: &[usize], cell: usize, stripes: usize,
                                stream: *mut c_void) -> Result<()> {
        let (k, m) = (self.data_units, self.parity_units);
        assert!(shards.len() == k + m && shard_strides.len() == k + m, "one slot per shard");
        assert!(out.len() == k && out_strides.len() == k, "one output slot per data shard");
        check(unsafe {
            hec_decode_device(self.raw, shards.as_ptr(), shard_strides.as_ptr(), out.as_ptr(), out_strides.as_ptr(),
                              cell, stripes, stream)
        })
    }

    /// Waits for `stream` (null = the default stream) on the coder's device.
    pub fn synchronize(&self, stream: *mut c_void) -> Result<()> {
        check(unsafe { hec_device_synchronize(self.device, stream) })
    }

    /// `Coder::encode` (gf256.rs:61-80): m freshly allocated parity shards.
    pub fn encode(&self, data: &[Bytes]) -> Vec<Bytes> {
        encode_raw(self.raw, self.data_units, self.parity_units, data)
    }

    /// `Coder::decode` (gf256.rs:84-137): rebuilds every missing data slot.
    pub fn decode(&self, data: &mut [Option<Bytes>]) -> Result<()> {
        decode_raw(self.raw, self.data_units, self.parity_units, data)
    }

    /// A whole file in file order (rows of k cells, the last one possibly
    /// short: `CellBuffer::write` / `encode`, block_writer.rs:791-851) ->
    /// `parity` = ceil(len / (k*cell)) rows of m cells; the short row's parity
    /// cells hold len(cell 0) bytes, zero past them.
    pub fn encode_file(&self, data: &[u8], cell: usize, parity: &mut [u8]) -> Result<()> {
        let (k, m) = (self.data_units, self.parity_units);
        assert!(cell > 0, "cell_len > 0");
        let rows = data.len().div_ceil(k * cell);
        assert!(parity.len() >= rows * m * cell, "parity holds ceil(len / row) * m cells");
        check(unsafe { hec_encode_rows_host(self.raw, data.as_ptr(), data.len(), parity.as_mut_ptr(), cell, 16) })
    }

    /// The blocks of one block group (`vertical[i]` = shard i's block, any
    /// length up to its `max_offset`; `None` = failed reader) -> the file's
    /// `file.len()` bytes, short and absent cells read as zeros
    /// (`CellReader::next_cell`, block_reader.rs:343-378).
    pub fn decode_file(&self, vertical: &[Option<&[u8]>], cell: usize, file: &mut [u8]) -> Result<()> {
        let (k, m) = (self.data_units, self.parity_units);
        assert_eq!(vertical.len(), k + m, "one slot per shard");
        assert!(cell > 0, "cell_len > 0");
        let ptrs: Vec<*const u8> = vertical.iter().map(|v| v.map_or(std::ptr::null(), |b| b.as_ptr())).collect();
        let lens: Vec<usize> = vertical.iter().map(|v| v.map_or(0, <[u8]>::len)).collect();
        check(unsafe {
            hec_decode_rows_host(self.raw, ptrs.as_ptr(), lens.as_ptr(), cell, file.as_mut_ptr(), file.len(), 16)
        })
    }

    /// N full rows in file order (row r = `rows[r*k*cell ..]`) -> N x m
    /// parity cells, one pinned H2D / encode / D2H pipeline instead of N
    /// `CellBuffer::encode` calls (block_writer.rs:838).
    pub fn encode_rows(&self, rows: &[u8], cell: usize, parity: &mut [u8]) -> Result<()> {
        let (k, m) = (self.data_units, self.parity_units);
        assert!(cell > 0 && rows.len() % (k * cell) == 0, "whole rows of k cells");
        let n = rows.len() / (k * cell);
        assert!(parity.len() >= n * m * cell, "parity holds n * m cells");
        check(unsafe { hec_encode_host_batch(self.raw, rows.as_ptr(), parity.as_mut_ptr(), cell, n, 16) })
    }

    /// Reader side: `vertical[i]` holds `n` consecutive cells of shard i
    /// (`None` = failed reader); `file` receives n rows of k cells in file
    /// order with lost cells rebuilt -- n `ec_decode` calls (ec/mod.rs:62-89).
    pub fn decode_rows(&self, vertical: &[Option<&[u8]>], cell: usize, n: usize, file: &mut [u8]) -> Result<()> {
        let (k, m) = (self.data_units, self.parity_units);
        assert_eq!(vertical.len(), k + m, "one slot per shard");
        assert!(cell > 0, "cell_len > 0");
        assert!(vertical.iter().flatten().all(|v| v.len() >= n * cell), "every shard holds n cells");
        assert!(file.len() >= n * k * cell, "file holds n rows");
        let ptrs: Vec<*const u8> = vertical.iter().map(|v| v.map_or(std::ptr::null(), |b| b.as_ptr())).collect();
        check(unsafe { hec_decode_host_batch(self.raw, ptrs.as_ptr(), cell, n, file.as_mut_ptr(), 16) })
    }

    /// Verified striped read of `rows` rows already on the device
    /// (`block_reader.rs:480-525` + `ReadPacket::get_data`): shard i of row r
    /// at `shards[i] + r * strides[i]` (null = no reader); `sums` holds the
    /// packets' checksums `[row][k+m][chunk]` big-endian.  Missing or failed
    /// data cells are rebuilt into `out[i]` (may be `shards[i]` itself: in-
    /// place repair); `bad[r*(k+m)+i] = 1` marks the cells that failed.
    ///
    /// # Safety
    /// Every pointer is a device pointer valid for the layout above, and the
    /// stream belongs to the coder's device.
    #[allow(clippy::too_many_arguments)]
    pub unsafe fn decode_verified(&self, checksum_type: i32, shards: &[*const u8], strides: &[usize],
                                  out: &[*mut u8], out_strides: &[usize], cell: usize, rows: usize,
                                  bytes_per_checksum: usize, sums: *const u8, bad: *mut u8,
                                  stream: *mut c_void) -> Result<()> {
        let (k, m) = (self.data_units, self.parity_units);
        assert!(shards.len() == k + m && strides.len() == k + m, "one slot per shard");
        assert!(out.len() == k && out_strides.len() == k, "one output slot per data shard");
        check(unsafe {
            hec_decode_verify_device(self.raw, checksum_type, shards.as_ptr(), strides.as_ptr(), out.as_ptr(),
                                     out_strides.as_ptr(), cell, rows, bytes_per_checksum, sums, bad, stream)
        })
    }
}

/// HBM on one device (`hec_device_alloc`), freed on drop: the stripe
/// buffers of `encode_device` / `decode_device` for a caller (the `mi355x`
/// Criterion group of rust/benches/ec.rs) with no HIP binding of its own.
pub struct DeviceBuffer {
    device: i32,
    ptr: *mut u8,
    len: usize,
}

unsafe impl Send for DeviceBuffer {}
unsafe impl Sync for DeviceBuffer {}

impl DeviceBuffer {
    pub fn new(device: i32, len: usize) -> Result<Self> {
        let mut p = std::ptr::null_mut();
        check(unsafe { hec_device_alloc(device, len, 0, &mut p) })?;
        Ok(Self { device, ptr: p.cast(), len })
    }

    /// A buffer holding a copy of `host`.
    pub fn upload(device: i32, host: &[u8]) -> Result<Self> {
        let b = Self::new(device, host.len())?;
        check(unsafe { hec_device_copy(device, b.ptr.cast(), host.as_ptr().cast(), host.len()) })?;
        Ok(b)
    }

    /// Copies the buffer into `host` (`host.len()` bytes from its start).
    pub fn download(&self, host: &mut [u8]) -> Result<()> {
        assert!(host.len() <= self.len, "read past the buffer");
        check(unsafe { hec_device_copy(self.device, host.as_mut_ptr().cast(), self.ptr.cast(), host.len()) })
    }

    /// Device address of byte `off`.
    pub fn at(&self, off: usize) -> *mut u8 {
        assert!(off <= self.len, "offset past the buffer");
        self.ptr.wrapping_add(off)
    }

    pub fn len(&self) -> usize {
        self.len
    }

    pub fn is_empty(&self) -> bool {
        self.len == 0
    }
}

impl Drop for DeviceBuffer {
    fn drop(&mut self) {
        unsafe { hec_device_free(self.device, self.ptr.cast()) };
    }
}

impl Drop for GpuCoder {
    fn drop(&mut self) {
        unsafe { hec_coder_destroy(self.raw) }
    }
}

fn encode_raw(raw: *mut HecCoder, k: usize, m: usize, data: &[Bytes]) -> Vec<Bytes> {
    assert_eq!(data.len(), k, "data.len() == data_units (gf256.rs:62)");
    let n = data[0].len();
    assert!(n > 0, "shards must not be empty (matrix.rs:57)");
    assert!(data.iter().all(|s| s.len() == n), "equal shard lengths (gf256.rs:65)");
    let mut parity: Vec<BytesMut> = (0..m).map(|_| BytesMut::zeroed(n)).collect();
    let ins: Vec<*const u8> = data.iter().map(|d| d.as_ptr()).collect();
    let outs: Vec<*mut u8> = parity.iter_mut().map(|p| p.as_mut_ptr()).collect();
    let rc = unsafe { hec_encode(raw, ins.as_ptr(), n, outs.as_ptr()) };
    // the reference encode cannot fail; a device error here is a bug or a lost GPU
    assert_eq!(rc, HEC_OK, "hec_encode: {}", err(rc));
    parity.into_iter().map(BytesMut::freeze).collect()
}

fn decode_raw(raw: *mut HecCoder, k: usize, m: usize, data: &mut [Option<Bytes>]) -> Result<()> {
    assert_eq!(data.len(), k + m, "data.len() == data_units + parity_units");
    if data.iter().take(k).all(Option::is_some) {
        return Ok(()); // gf256.rs:102-105
    }
    let n = match data.iter().flatten().next() {
        Some(b) => b.len(),
        None => return Err(err(HEC_ERR_NOT_ENOUGH_SHARDS)),
    };
    // the engine reads n bytes from each of the first k present shards (the
    // survivors it decodes from): hold the reference's equal-length
    // precondition over exactly those (matrix.rs:212-216 asserts it over the
    // k selected rows only; a longer or shorter shard past them is not read)
    assert!(n > 0, "shards must not be empty (matrix.rs:57)");
    assert!(data.iter().flatten().take(k).all(|b| b.len() == n), "equal shard lengths (matrix.rs:215)");
    let ins: Vec<*const u8> = data.iter().map(|d| d.as_ref().map_or(std::ptr::null(), |b| b.as_ptr())).collect();
    let mut rec: Vec<Option<BytesMut>> =
        (0..k + m).map(|i| (i < k && data[i].is_none()).then(|| BytesMut::zeroed(n))).collect();
    // parity slots (and present data slots) pass null: never written
    let outs: Vec<*mut u8> =
        rec.iter_mut().map(|r| r.as_mut().map_or(std::ptr::null_mut(), |b| b.as_mut_ptr())).collect();
    check(unsafe { hec_decode(raw, ins.as_ptr(), n, outs.as_ptr()) })?;
    for (i, r) in rec.into_iter().enumerate() {
        if let Some(b) = r {
            data[i] = Some(b.freeze());
        }
    }
    Ok(())
}

/// The engine coder behind the reference's `Coder` when the `mi355x` feature
/// forwards it (rust/patches/ec_mi355x.patch): `Coder::new` acquires one from
/// the process-wide pool, drop releases it.  `Coder::new` runs per decoded
/// row (ec/mod.rs:71) and per block writer (block_writer.rs:787), so a pool
/// hit costs a mutex and a vector pop -- no streams, events or buffers are
/// created (`tests/cpp/shim_replay.c` times 10,000 cycles).  The device is
/// `HDFS_EC_AMD_DEVICE` if set, else any (round-robin over the visible GPUs;
/// an engine host-only coder, `HEC_DEVICE_HOST`, when none is visible).  When
/// the device coder cannot be had (a bad `HDFS_EC_AMD_DEVICE`, device memory
/// exhausted) `acquire` falls back to a host-only coder, so only a library
/// that cannot allocate at all returns an error -- which the patched
/// `Coder::new` turns into its reference CPU path.
/// Rows below the coder's host limit are coded on the calling thread.
pub struct PooledCoder {
    raw: *mut HecCoder,
    data_units: usize,
    parity_units: usize,
}

unsafe impl Send for PooledCoder {}
unsafe impl Sync for PooledCoder {}

impl PooledCoder {
    pub fn acquire(codec: &str, data_units: usize, parity_units: usize) -> Result<Self> {
        assert_eq!(unsafe { hec_abi_version() }, ABI_VERSION, "libhdfs_ec_amd ABI mismatch");
        let device: i32 =
            std::env::var("HDFS_EC_AMD_DEVICE").ok().and_then(|v| v.parse().ok()).unwrap_or(-1);
        let name = std::ffi::CString::new(codec).map_err(|_| HdfsError::InvalidArgument(codec.to_string()))?;
        let mut raw = std::ptr::null_mut();
        let rc = unsafe { hec_coder_acquire(name.as_ptr(), data_units, parity_units, device, &mut raw) };
        if rc != HEC_OK {
            if rc == HEC_ERR_INVALID_ARG || rc == HEC_ERR_UNSUPPORTED_CODEC {
                return Err(err(rc));
            }
            log::warn!("MI355X EC engine: device coder unavailable ({}), host-only coder", err(rc));
            check(unsafe { hec_coder_acquire(name.as_ptr(), data_units, parity_units, HEC_DEVICE_HOST, &mut raw) })?;
        }
        Ok(Self { raw, data_units, parity_units })
    }

    /// True when this coder runs on the engine's host routine (no GPU).
    pub fn host_only(&self) -> bool {
        unsafe { hec_coder_device(self.raw) == HEC_DEVICE_HOST }
    }

    pub fn encode(&self, data: &[Bytes]) -> Vec<Bytes> {
        encode_raw(self.raw, self.data_units, self.parity_units, data)
    }

    pub fn decode(&self, data: &mut [Option<Bytes>]) -> Result<()> {
        decode_raw(self.raw, self.data_units, self.parity_units, data)
    }
}

impl Drop for PooledCoder {
    fn drop(&mut self) {
        unsafe { hec_coder_release(self.raw) }
    }
}

/// All GPUs of a node from one client process: a batch split into
/// contiguous stripe ranges, one device and host thread each, no collective
/// (stripes are independent).
pub struct GpuGroup {
    raw: *mut HecGroup,
    data_units: usize,
    parity_units: usize,
}

unsafe impl Send for GpuGroup {}
unsafe impl Sync for GpuGroup {}

impl GpuGroup {
    pub fn new(codec: &str, data_units: usize, parity_units: usize, devices: &[i32]) -> Result<Self> {
        assert_eq!(unsafe { hec_abi_version() }, ABI_VERSION, "libhdfs_ec_amd ABI mismatch");
        let name = std::ffi::CString::new(codec).map_err(|_| HdfsError::InvalidArgument(codec.to_string()))?;
        let mut raw = std::ptr::null_mut();
        check(unsafe {
            hec_group_create(name.as_ptr(), data_units, parity_units, devices.as_ptr(), devices.len(), &mut raw)
        })?;
        Ok(Self { raw, data_units, parity_units })
    }

    /// `GpuCoder::encode_rows` across every GPU of the group.
    pub fn encode_rows(&self, rows: &[u8], cell: usize, parity: &mut [u8]) -> Result<()> {
        let (k, m) = (self.data_units, self.parity_units);
        assert!(cell > 0 && rows.len() % (k * cell) == 0, "whole rows of k cells");
        let n = rows.len() / (k * cell);
        assert!(parity.len() >= n * m * cell, "parity holds n * m cells");
        check(unsafe { hec_group_encode_host_batch(self.raw, rows.as_ptr(), parity.as_mut_ptr(), cell, n, 16) })
    }

    /// `GpuCoder::decode_rows` across every GPU of the group.
    pub fn decode_rows(&self, vertical: &[Option<&[u8]>], cell: usize, n: usize, file: &mut [u8]) -> Result<()> {
        let (k, m) = (self.data_units, self.parity_units);
        assert_eq!(vertical.len(), k + m, "one slot per shard");
        assert!(vertical.iter().flatten().all(|v| v.len() >= n * cell), "every shard holds n cells");
        assert!(file.len() >= n * k * cell, "file holds n rows");
        let ptrs: Vec<*const u8> = vertical.iter().map(|v| v.map_or(std::ptr::null(), |b| b.as_ptr())).collect();
        check(unsafe { hec_group_decode_host_batch(self.raw, ptrs.as_ptr(), cell, n, file.as_mut_ptr(), 16) })
    }
}

impl Drop for GpuGroup {
    fn drop(&mut self) {
        unsafe { hec_group_destroy(self.raw) }
    }
}

//! Row-batched cell buffer for the striped writer, used in place of the
//! reference's `CellBuffer` (`rust/src/hdfs/block_writer.rs:770-851`) when the
//! `mi355x` feature is on (rust/patches/ec_mi355x.patch).
//!
//! The reference encodes one row (k cells) per `Coder::encode` call and hands
//! each block writer one cell.  GF(2^8) coding is bytewise, so `r` consecutive
//! cells of shard i laid back to back (a "vertical stripe", the layout
//! `EcSchema::ec_decode` already takes on the read side, `ec/mod.rs:62-89`)
//! encode in ONE call to the same parity bytes, back to back.  This buffer
//! therefore collects up to `ROWS_PER_CALL` rows per shard before encoding:
//! one engine call (one pipelined PCIe round trip, or one host-routine pass)
//! per `ROWS_PER_CALL` rows instead of one per row.  Each block writer then
//! receives its cells of those rows as one buffer -- the same byte stream the
//! reference writes cell by cell.
//!
//! Semantics kept from the reference:
//!   * cells fill in order (cell 0 of a row before cell 1, `:791-806`);
//!   * a short last row is zero-padded to the length of its cell 0 for the
//!     encode, its parity cells are that long, and the data cells are written
//!     at their original lengths (`:817-851`) -- it is coded in a second call
//!     after the whole rows;
//!   * an empty shard stream is skipped by `write_cells` (no block created).
//!
//! Written for hdfs-native 0.14.1; not compiled in this repository (no cargo).
//! `tests/cpp/shim_replay.c` replays the resulting engine calls against the
//! oracle.

use bytes::{BufMut, Bytes, BytesMut};

use crate::ec::{EcSchema, gf256::Coder};

/// Rows buffered per encode (and per decode on the read side): 4 x k cells,
/// 24 MiB of data for RS(6,3) with 1 MiB cells.
pub(crate) const ROWS_PER_CALL: usize = 4;

pub(crate) struct CellBuffer {
    /// shard i: its cells of the buffered rows, back to back
    buffers: Vec<BytesMut>,
    cell_size: usize,
    parity_units: usize,
    /// shard receiving bytes in the current (incomplete) row
    current_index: usize,
    /// complete rows buffered
    rows: usize,
    coder: Coder,
}

impl CellBuffer {
    pub(crate) fn new(ec_schema: &EcSchema) -> Self {
        let buffers = (0..ec_schema.data_units)
            .map(|_| BytesMut::with_capacity(ROWS_PER_CALL * ec_schema.cell_size))
            .collect();
        Self {
            buffers,
            cell_size: ec_schema.cell_size,
            parity_units: ec_schema.parity_units,
            current_index: 0,
            rows: 0,
            coder: Coder::new(ec_schema.data_units, ec_schema.parity_units),
        }
    }

    pub(crate) fn write(&mut self, buf: &mut Bytes) {
        while !buf.is_empty() && !self.is_full() {
            // this shard's cell of the current row ends here
            let cell_end = (self.rows + 1) * self.cell_size;
            let current_buffer = &mut self.buffers[self.current_index];
            let split_at = usize::min(cell_end - current_buffer.len(), buf.len());
            current_buffer.put(buf.split_to(split_at));
            if current_buffer.len() == cell_end {
                self.current_index += 1;
                if self.current_index == self.buffers.len() {
                    self.current_index = 0;
                    self.rows += 1;
                }
            }
        }
    }

    #[inline]
    pub(crate) fn is_full(&self) -> bool {
        self.rows == ROWS_PER_CALL
    }

    #[inline]
    pub(crate) fn is_empty(&self) -> bool {
        self.buffers[0].is_empty()
    }

    /// The k data streams (original lengths) followed by the m parity streams
    /// of the buffered rows; empties the buffer.
    pub(crate) fn encode(&mut self) -> Vec<Bytes> {
        let whole = self.rows * self.cell_size;
        // shard 0 is the longest: whole rows + the partial row's cell 0
        let slice_size = self.buffers[0].len();
        let original_sizes: Vec<usize> = self.buffers.iter().map(BytesMut::len).collect();

        let mut data: Vec<Bytes> = self
            .buffers
            .iter()
            .cloned()
            .map(|mut buf| {
                buf.resize(slice_size, 0);
                buf.freeze()
            })
            .collect();

        let mut parity: Vec<BytesMut> = (0..self.parity_units).map(|_| BytesMut::with_capacity(slice_size)).collect();
        // whole rows in one call, then the zero-padded partial row (if any)
        for (a, b) in [(0, whole), (whole, slice_size)] {
            if b > a {
                let part: Vec<Bytes> = data.iter().map(|d| d.slice(a..b)).collect();
                for (dst, src) in parity.iter_mut().zip(self.coder.encode(&part)) {
                    dst.put(src);
                }
            }
        }

        for (slice, size) in data.iter_mut().zip(original_sizes) {
            let _ = slice.split_off(size);
        }
        for buf in self.buffers.iter_mut() {
            buf.clear();
        }
        self.current_index = 0;
        self.rows = 0;

        data.extend(parity.into_iter().map(BytesMut::freeze));
        data
    }
}

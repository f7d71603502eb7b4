//! `scan_file`: a whole-file scan -> one `Canonical` per column, through ONE engine plan.
//!
//! The reference scans a file with `LayoutBatchStream` (vortex-serde/src/layouts/read/
//! stream.rs:91): per chunk it reads the column messages, builds `ArrayView`s, swizzles them into a
//! `StructArray`, and a caller canonicalizes each field with `struct_to_arrow`
//! (vortex-array/src/canonical.rs:169-187); a field that spans chunks is a `ChunkedArray`
//! whose canonicalize packs the chunks (array/chunked/canonical.rs:16-25, 129-148).  Going
//! through `GpuEncoding` on those in-memory arrays works but uploads every buffer separately
//! (flatten.rs) and returns one chunk at a time.  Here the engine's own reader does it the
//! MI355X way (include/vortex_file.h):
//!
//! 1. `vxg_file_open` parses EOF / Postscript / Footer / layouts from the file bytes (host);
//! 2. per column, the byte range of its chunks' messages is copied to HBM with ONE copy
//!    (`vxg_alloc` + `vxg_memcpy_h2d`) and `vxg_file_column_array` builds its ChunkedArray
//!    descriptor tree over that device region (buffers resolved in place, no per-buffer copies);
//! 3. the outputs are sized with `vxg_canonical_layout` and allocated in HBM;
//! 4. `vxg_plan_create` records the canonicalize of every column as one HIP graph (batched
//!    launches across columns), `vxg_plan_launch` runs it, `vxg_stream_sync` reports errors;
//! 5. every output is copied into pinned host memory and handed to Vortex as zero-copy Arrow
//!    buffers (canonical.rs), the device memory released.
//!
//! An Extension column (e.g. `vortex.date`) comes back as the canonical array of its storage
//! dtype, which is what `ExtensionArray::storage` canonicalizes to.
//!
//! UNTESTED (no Rust toolchain in this image): `tests/test_gpu_file.py` exercises the same call
//! sequence through the Python binding (`vortex_amd/file.py`: VortexFile, DeviceColumns, Plan).

use std::ffi::{c_void, CStr};
use std::ops::Range;
use std::ptr;

use arrow_buffer::{BooleanBuffer, Buffer as ArrowBuffer};
use vortex::array::{BoolArray, PrimitiveArray, VarBinViewArray};
use vortex::Canonical;
use vortex_buffer::Buffer;
use vortex_dtype::{DType, Nullability};
use vortex_error::{vortex_bail, vortex_err, VortexResult};

use crate::canonical::{bytes_array, to_host, validity};
use crate::meta::ptype_of_code;
use crate::{check, ffi, GpuSession};

/// A parsed Vortex file (`vxg_file`) over host bytes that outlive it.
pub struct GpuFile<'b> {
    raw: *mut ffi::vxg_file,
    bytes: &'b [u8],
}

impl Drop for GpuFile<'_> {
    fn drop(&mut self) {
        unsafe {
            ffi::vxg_file_close(self.raw);
        }
    }
}

/// One column of the file's Struct schema.
#[derive(Clone, Debug)]
pub struct ColumnInfo {
    pub name: String,
    pub dtype: DType,
    pub n_chunks: u32,
    pub rows: u64,
    pub extension_id: Option<String>,
}

impl<'b> GpuFile<'b> {
    pub fn open(bytes: &'b [u8]) -> VortexResult<Self> {
        let mut raw = ptr::null_mut();
        check(unsafe { ffi::vxg_file_open(bytes.as_ptr().cast(), bytes.len() as u64, &mut raw) })?;
        Ok(Self { raw, bytes })
    }

    pub fn row_count(&self) -> VortexResult<u64> {
        let (mut rows, mut n) = (0u64, 0u32);
        check(unsafe { ffi::vxg_file_info(self.raw, &mut rows, &mut n) })?;
        Ok(rows)
    }

    pub fn columns(&self) -> VortexResult<Vec<ColumnInfo>> {
        let (mut rows, mut n) = (0u64, 0u32);
        check(unsafe { ffi::vxg_file_info(self.raw, &mut rows, &mut n) })?;
        (0..n).map(|c| self.column(c)).collect()
    }

    fn column(&self, c: u32) -> VortexResult<ColumnInfo> {
        let mut ci: ffi::vxg_file_column = unsafe { std::mem::zeroed() };
        check(unsafe { ffi::vxg_file_column_info(self.raw, c, &mut ci) })?;
        let name = unsafe { CStr::from_ptr(ci.name) }.to_string_lossy().into_owned();
        let nullability = if ci.nullable != 0 { Nullability::Nullable } else { Nullability::NonNullable };
        let dtype = match u32::from(ci.dtype) {
            d if d == ffi::VXG_DTYPE_PRIMITIVE as u32 => DType::Primitive(ptype_of_code(ci.ptype)?, nullability),
            d if d == ffi::VXG_DTYPE_BOOL as u32 => DType::Bool(nullability),
            d if d == ffi::VXG_DTYPE_UTF8 as u32 => DType::Utf8(nullability),
            d if d == ffi::VXG_DTYPE_BINARY as u32 => DType::Binary(nullability),
            other => vortex_bail!(NotImplemented: format!("scan of dtype code {}", other), "vortex-gpu"),
        };
        let extension_id = if ci.extension_id.is_null() {
            None
        } else {
            Some(unsafe { CStr::from_ptr(ci.extension_id) }.to_string_lossy().into_owned())
        };
        Ok(ColumnInfo { name, dtype, n_chunks: ci.n_chunks, rows: ci.rows, extension_id })
    }

    /// File byte range covering the messages of chunks `chunks` of column `c` (the messages of a
    /// column are written consecutively; the range is the union either way).
    fn byte_range(&self, c: u32, chunks: &Range<u32>) -> VortexResult<(u64, u64)> {
        let (mut lo, mut hi) = (u64::MAX, 0u64);
        for k in chunks.clone() {
            let mut ch: ffi::vxg_file_chunk = unsafe { std::mem::zeroed() };
            check(unsafe { ffi::vxg_file_chunk_info(self.raw, c, k, &mut ch) })?;
            lo = lo.min(ch.message_begin);
            hi = hi.max(ch.message_end);
        }
        if lo > hi || hi > self.bytes.len() as u64 {
            vortex_bail!(InvalidSerde: "chunk messages outside the file");
        }
        Ok((lo, hi))
    }
}

/// Device memory owned by a scan (regions, chunk offsets, outputs).
struct DeviceAllocs<'s> {
    session: &'s GpuSession,
    ptrs: Vec<*mut c_void>,
}

impl DeviceAllocs<'_> {
    fn alloc(&mut self, bytes: u64) -> VortexResult<*mut c_void> {
        let mut d = ptr::null_mut();
        check(unsafe { ffi::vxg_alloc(self.session.raw(), bytes.max(16), &mut d) })?;
        self.ptrs.push(d);
        Ok(d)
    }
}

impl Drop for DeviceAllocs<'_> {
    fn drop(&mut self) {
        for &p in &self.ptrs {
            unsafe {
                ffi::vxg_free(self.session.raw(), p);
            }
        }
    }
}

struct Plan(*mut ffi::vxg_plan);

impl Drop for Plan {
    fn drop(&mut self) {
        unsafe {
            ffi::vxg_plan_destroy(self.0);
        }
    }
}

/// Canonicalize chunks `chunks` (all if None) of every column (or the given ones) of the Vortex
/// file in `bytes`: `Vec<(column name, Canonical)>` in schema order, decoded on the GPU by one
/// plan.  The file bytes are read once per column range (one H2D copy each).
pub fn scan_file(
    session: &GpuSession,
    bytes: &[u8],
    columns: Option<&[u32]>,
    chunks: Option<Range<u32>>,
) -> VortexResult<Vec<(String, Canonical)>> {
    let file = GpuFile::open(bytes)?;
    let infos = file.columns()?;
    let selected: Vec<u32> = match columns {
        Some(c) => c.to_vec(),
        None => (0..infos.len() as u32).collect(),
    };
    let mut dev = DeviceAllocs { session, ptrs: Vec::new() };
    let mut nodes: Vec<ffi::vxg_array> = Vec::with_capacity(selected.len());
    for &c in &selected {
        let info = infos.get(c as usize).ok_or_else(|| vortex_err!(OutOfBounds: c as usize, 0, infos.len()))?;
        let range = chunks.clone().unwrap_or(0..info.n_chunks);
        if range.start >= range.end || range.end > info.n_chunks {
            vortex_bail!(InvalidArgument: "chunk range {:?} of a column with {} chunks", range, info.n_chunks);
        }
        // (2) one H2D copy of the column's message range + its chunk offsets
        let (lo, hi) = file.byte_range(c, &range)?;
        let region = dev.alloc(hi - lo)?;
        check(unsafe {
            ffi::vxg_memcpy_h2d(session.raw(), region, bytes[lo as usize..].as_ptr().cast(), hi - lo, ptr::null_mut())
        })?;
        let mut offs = vec![0u64; (range.end - range.start + 1) as usize];
        check(unsafe { ffi::vxg_file_chunk_offsets(file.raw, c, range.start, range.end, offs.as_mut_ptr()) })?;
        let offs_dev = dev.alloc(8 * offs.len() as u64)?;
        check(unsafe {
            ffi::vxg_memcpy_h2d(session.raw(), offs_dev, offs.as_ptr().cast(), 8 * offs.len() as u64, ptr::null_mut())
        })?;
        let mut node: *const ffi::vxg_array = ptr::null();
        check(unsafe {
            ffi::vxg_file_column_array(file.raw, c, range.start, range.end, region, lo, hi - lo, offs_dev, &mut node)
        })?;
        // SAFETY: the tree is owned by `file`, which outlives the plan below
        nodes.push(unsafe { *node });
    }
    // (3) outputs in HBM, sized by the engine
    let mut outs: Vec<ffi::vxg_canonical> = vec![unsafe { std::mem::zeroed() }; nodes.len()];
    let mut tables: Vec<Vec<ffi::vxg_data_buffer>> = Vec::with_capacity(nodes.len());
    for (node, out) in nodes.iter().zip(outs.iter_mut()) {
        let (mut vb, mut db, mut nb) = (0u64, 0u64, 0u32);
        check(unsafe { ffi::vxg_canonical_layout(session.raw(), node, &mut vb, &mut db, ptr::null_mut(), 0, &mut nb) })?;
        let mut table = vec![ffi::vxg_data_buffer { offset: 0, len: 0 }; nb.max(1) as usize];
        if nb > 1 {
            check(unsafe {
                ffi::vxg_canonical_layout(session.raw(), node, &mut vb, &mut db, table.as_mut_ptr(), nb, &mut nb)
            })?;
        }
        let string = u32::from(node.dtype) == ffi::VXG_DTYPE_UTF8 as u32 || u32::from(node.dtype) == ffi::VXG_DTYPE_BINARY as u32;
        if string {
            out.views = dev.alloc(vb)?;
            out.data = dev.alloc(db + 16)?;
            out.data_bytes = db;
            out.data_buffers = table.as_mut_ptr();
            out.n_data_buffers = nb;
            out.data_buffers_cap = table.len() as u32;
        } else {
            out.values = dev.alloc(vb)?;
        }
        if node.nullable != 0 {
            out.validity = dev.alloc(((node.len + 31) / 32) * 4 + 4)?;
        }
        tables.push(table);
    }
    // (4) one plan for every column; launched once, so recorded without VXG_PLAN_MEASURE (create
    // executes nothing and picks batched/unbatched by the plan's output size)
    let mut raw_plan = ptr::null_mut();
    check(unsafe {
        ffi::vxg_plan_create(session.raw(), nodes.as_ptr(), outs.as_mut_ptr(), nodes.len() as u32, &mut raw_plan)
    })?;
    let plan = Plan(raw_plan);
    check(unsafe { ffi::vxg_plan_launch(plan.0, ptr::null_mut()) })?;
    check(unsafe { ffi::vxg_stream_sync(session.raw(), ptr::null_mut()) })?;
    // (5) host Arrow buffers
    let mut result = Vec::with_capacity(selected.len());
    for ((&c, out), table) in selected.iter().zip(&outs).zip(&tables) {
        let info = &infos[c as usize];
        let len = out.len as usize;
        let vbits = (out.len + 31) / 32 * 4;
        let valid = if out.validity.is_null() { None } else { Some(to_host(session, out.validity, vbits)?) };
        let canonical = match &info.dtype {
            DType::Primitive(p, _) => {
                let v = to_host(session, out.values, (len * p.byte_width()) as u64)?;
                check(unsafe { ffi::vxg_stream_sync(session.raw(), ptr::null_mut()) })?;
                Canonical::Primitive(PrimitiveArray::new(Buffer::from(v), *p, validity(&info.dtype, valid, len)?))
            }
            DType::Bool(_) => {
                let v = to_host(session, out.values, vbits)?;
                check(unsafe { ffi::vxg_stream_sync(session.raw(), ptr::null_mut()) })?;
                Canonical::Bool(BoolArray::try_new(BooleanBuffer::new(v, 0, len), validity(&info.dtype, valid, len)?)?)
            }
            _ => {
                let views = to_host(session, out.views, 16 * out.len)?;
                let data: ArrowBuffer = to_host(session, out.data, out.data_bytes)?;
                check(unsafe { ffi::vxg_stream_sync(session.raw(), ptr::null_mut()) })?;
                let buffers = table[..out.n_data_buffers as usize]
                    .iter()
                    .map(|b| bytes_array(data.slice_with_length(b.offset as usize, b.len as usize)))
                    .collect::<Vec<_>>();
                Canonical::VarBinView(VarBinViewArray::try_new(
                    bytes_array(views),
                    buffers,
                    info.dtype.clone(),
                    validity(&info.dtype, valid, len)?,
                )?)
            }
        };
        result.push((info.name.clone(), canonical));
    }
    drop(plan);
    Ok(result)
}

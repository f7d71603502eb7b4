//! `vxg_canonical` -> Vortex `Canonical` (vortex-array/src/canonical.rs:56-63).
//!
//! The engine allocates the outputs in HBM (the descriptor's device pointers left NULL); each is
//! copied into pinned host memory (`vxg_host_alloc`) and handed to Vortex without another copy
//! as an Arrow buffer that owns the pinned allocation (`Buffer::from_custom_allocation`), then
//! the device outputs are released.  Bool values and validity are LSB bitmaps of `len` bits
//! (arrow BooleanBuffer); VarBinView outputs are the views plus one data buffer per chunk, all
//! inside one `data` allocation (`vxg_canonical.data_buffers`), like pack_views
//! (array/chunked/canonical.rs:194-236).

use std::ffi::c_void;
use std::ptr::{self, NonNull};
use std::sync::Arc;

use arrow_buffer::{BooleanBuffer, Buffer as ArrowBuffer};
use vortex::array::{BoolArray, PrimitiveArray, VarBinViewArray};
use vortex::validity::Validity;
use vortex::{Array, ArrayDType, Canonical, IntoArray};
use vortex_buffer::Buffer;
use vortex_dtype::{DType, PType};
use vortex_error::{vortex_bail, vortex_err, VortexResult};

use crate::flatten::DeviceTree;
use crate::{check, ffi, GpuSession};

/// Pinned host memory owned by an Arrow buffer; freed when the last buffer slice drops.  The
/// session that allocated it must outlive it (the global session lives for the process).
struct PinnedHost {
    ctx: *mut ffi::vxg_ctx,
    ptr: *mut c_void,
}

// SAFETY: the allocation is plain host memory; vxg_host_free is thread-safe.
unsafe impl Send for PinnedHost {}
unsafe impl Sync for PinnedHost {}

impl Drop for PinnedHost {
    fn drop(&mut self) {
        unsafe {
            ffi::vxg_host_free(self.ctx, self.ptr);
        }
    }
}

/// Device outputs the engine allocated: released after the copies.
struct DeviceOutputs {
    ctx: *mut ffi::vxg_ctx,
    ptrs: Vec<*mut c_void>,
}

impl Drop for DeviceOutputs {
    fn drop(&mut self) {
        for &p in &self.ptrs {
            if !p.is_null() {
                unsafe {
                    ffi::vxg_free(self.ctx, p);
                }
            }
        }
    }
}

pub(crate) fn to_host(s: &GpuSession, dptr: *mut c_void, bytes: u64) -> VortexResult<ArrowBuffer> {
    let mut h = ptr::null_mut();
    check(unsafe { ffi::vxg_host_alloc(s.raw(), bytes.max(1), &mut h) })?;
    let owner = Arc::new(PinnedHost { ctx: s.raw(), ptr: h });
    if bytes > 0 {
        check(unsafe { ffi::vxg_memcpy_d2h(s.raw(), h, dptr, bytes, ptr::null_mut()) })?;
    }
    let nn = NonNull::new(h.cast::<u8>()).ok_or_else(|| vortex_err!(ComputeError: "null pinned allocation"))?;
    // SAFETY: `h` points at `bytes` bytes kept alive by `owner`; the copy completes before the
    // buffer is read (stream sync in `canonicalize`).
    Ok(unsafe { ArrowBuffer::from_custom_allocation(nn, bytes as usize, owner) })
}

pub(crate) fn validity(dtype: &DType, bits: Option<ArrowBuffer>, len: usize) -> VortexResult<Validity> {
    if !dtype.is_nullable() {
        return Ok(Validity::NonNullable);
    }
    Ok(match bits {
        None => Validity::AllValid,
        Some(b) => Validity::Array(BoolArray::try_new(BooleanBuffer::new(b, 0, len), Validity::NonNullable)?.into_array()),
    })
}

pub(crate) fn bytes_array(b: ArrowBuffer) -> Array {
    PrimitiveArray::new(Buffer::from(b), PType::U8, Validity::NonNullable).into_array()
}

pub(crate) fn canonicalize(s: &GpuSession, array: &Array) -> VortexResult<Canonical> {
    let tree = DeviceTree::new(s, array)?;
    let len = array.len();
    let mut out: ffi::vxg_canonical = unsafe { std::mem::zeroed() };
    // string outputs: the engine fills the data-buffer table (one entry per chunk)
    let mut table: Vec<ffi::vxg_data_buffer> = Vec::new();
    if matches!(array.dtype(), DType::Utf8(_) | DType::Binary(_)) {
        let (mut vb, mut db, mut nb) = (0u64, 0u64, 0u32);
        check(unsafe {
            ffi::vxg_canonical_layout(s.raw(), &tree.root, &mut vb, &mut db, ptr::null_mut(), 0, &mut nb)
        })?;
        table.resize(nb.max(1) as usize, ffi::vxg_data_buffer { offset: 0, len: 0 });
        out.data_buffers = table.as_mut_ptr();
        out.data_buffers_cap = table.len() as u32;
    }
    check(unsafe { ffi::vxg_canonicalize(s.raw(), &tree.root, &mut out, ptr::null_mut()) })?;
    let _device = DeviceOutputs { ctx: s.raw(), ptrs: vec![out.values, out.views, out.data, out.validity] };
    let vbits = (((len as u64) + 31) / 32) * 4;
    let values = if out.values.is_null() { None } else { Some(to_host(s, out.values, out.values_bytes)?) };
    let views = if out.views.is_null() { None } else { Some(to_host(s, out.views, 16 * len as u64)?) };
    let data = if out.data.is_null() { None } else { Some(to_host(s, out.data, out.data_bytes)?) };
    let valid = if out.validity.is_null() { None } else { Some(to_host(s, out.validity, vbits)?) };
    check(unsafe { ffi::vxg_stream_sync(s.raw(), ptr::null_mut()) })?;
    let validity = validity(array.dtype(), valid, len)?;

    match array.dtype() {
        DType::Primitive(p, _) => {
            let v = values.ok_or_else(|| vortex_err!(ComputeError: "engine returned no values"))?;
            let bytes = len * p.byte_width();
            Ok(Canonical::Primitive(PrimitiveArray::new(Buffer::from(v.slice_with_length(0, bytes)), *p, validity)))
        }
        DType::Bool(_) => {
            let v = values.ok_or_else(|| vortex_err!(ComputeError: "engine returned no values"))?;
            Ok(Canonical::Bool(BoolArray::try_new(BooleanBuffer::new(v, 0, len), validity)?))
        }
        DType::Utf8(_) | DType::Binary(_) => {
            let views = views.ok_or_else(|| vortex_err!(ComputeError: "engine returned no views"))?;
            let data = data.unwrap_or_else(|| ArrowBuffer::from_vec(Vec::<u8>::new()));
            let buffers = table[..out.n_data_buffers as usize]
                .iter()
                .map(|b| bytes_array(data.slice_with_length(b.offset as usize, b.len as usize)))
                .collect::<Vec<_>>();
            Ok(Canonical::VarBinView(VarBinViewArray::try_new(
                bytes_array(views.slice_with_length(0, 16 * len)),
                buffers,
                array.dtype().clone(),
                validity,
            )?))
        }
        other => vortex_bail!(NotImplemented: format!("GPU canonical output for {}", other), "vortex-gpu"),
    }
}

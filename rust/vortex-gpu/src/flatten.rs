//! Array tree -> `vxg_array` descriptors over device copies of the buffers.
//!
//! The descriptor tree mirrors the array tree node for node in the reference's child order
//! (`Array::children`, vortex-array/src/lib.rs:110-116, which for an `ArrayView` is the
//! encoding's visitor order, view.rs:150-156 -- the order the flatbuffer stores).  Each node's
//! metadata is its flexbuffer bytes (`ArrayView::metadata`, or `try_serialize_metadata` of an
//! in-memory `ArrayData`) converted by `meta::convert`.  Host buffers are copied into HBM once
//! per call; the copies and the descriptor arrays live as long as the `DeviceTree`.

use std::ffi::c_void;
use std::ptr;
use std::sync::Arc;

use vortex::{Array, ArrayDType, TrySerializeArrayMetadata};
use vortex_dtype::DType;
use vortex_error::{vortex_bail, VortexResult};

use crate::meta::{convert, ptype_code};
use crate::{check, ffi, GpuSession};

pub(crate) struct DeviceTree<'s> {
    session: &'s GpuSession,
    allocs: Vec<*mut c_void>,
    nodes: Vec<Box<[ffi::vxg_array]>>,
    buffers: Vec<Box<[ffi::vxg_buffer]>>,
    pub(crate) root: ffi::vxg_array,
}

impl Drop for DeviceTree<'_> {
    fn drop(&mut self) {
        for &p in &self.allocs {
            unsafe {
                ffi::vxg_free(self.session.raw(), p);
            }
        }
    }
}

/// (VXG_DTYPE_*, ptype code, nullable) of a dtype the engine decodes.
pub(crate) fn dtype_codes(dtype: &DType) -> VortexResult<(u8, u8, bool)> {
    Ok(match dtype {
        DType::Bool(n) => (ffi::VXG_DTYPE_BOOL as u8, 0, (*n).into()),
        DType::Primitive(p, n) => (ffi::VXG_DTYPE_PRIMITIVE as u8, ptype_code(*p), (*n).into()),
        DType::Utf8(n) => (ffi::VXG_DTYPE_UTF8 as u8, 0, (*n).into()),
        DType::Binary(n) => (ffi::VXG_DTYPE_BINARY as u8, 0, (*n).into()),
        DType::Null => (ffi::VXG_DTYPE_NULL as u8, 0, true),
        _ => vortex_bail!(NotImplemented: format!("GPU canonicalize of {}", dtype), "vortex-gpu"),
    })
}

fn metadata_bytes(a: &Array) -> VortexResult<Option<Arc<[u8]>>> {
    Ok(match a {
        Array::View(v) => v.metadata().map(Arc::from),
        Array::Data(d) => Some(d.metadata().try_serialize_metadata()?),
    })
}

impl<'s> DeviceTree<'s> {
    /// Flatten `array` (all its buffers copied to the device on the legacy default stream,
    /// which the engine's calls on that stream are ordered after).
    pub(crate) fn new(session: &'s GpuSession, array: &Array) -> VortexResult<Self> {
        let mut t = DeviceTree {
            session,
            allocs: Vec::new(),
            nodes: Vec::new(),
            buffers: Vec::new(),
            root: unsafe { std::mem::zeroed() },
        };
        t.root = t.node(array)?;
        Ok(t)
    }

    fn upload(&mut self, bytes: &[u8]) -> VortexResult<*const c_void> {
        let mut d = ptr::null_mut();
        check(unsafe { ffi::vxg_alloc(self.session.raw(), bytes.len() as u64, &mut d) })?;
        self.allocs.push(d);
        if !bytes.is_empty() {
            check(unsafe {
                ffi::vxg_memcpy_h2d(
                    self.session.raw(),
                    d,
                    bytes.as_ptr().cast(),
                    bytes.len() as u64,
                    ptr::null_mut(),
                )
            })?;
        }
        Ok(d)
    }

    fn node(&mut self, a: &Array) -> VortexResult<ffi::vxg_array> {
        let code = a.encoding().id().code();
        let (kind, ptype, nullable) = dtype_codes(a.dtype())?;
        let children = a.children();
        let md = metadata_bytes(a)?;
        let (meta, validity) = convert(code, a.dtype(), md.as_deref(), children.len())?;
        let mut n: ffi::vxg_array = unsafe { std::mem::zeroed() };
        n.encoding = code;
        n.dtype = kind;
        n.ptype = ptype;
        n.nullable = nullable as u8;
        n.validity = validity;
        n.len = a.len() as u64;
        n.meta = meta;
        if let Some(buf) = a.buffer() {
            let p = self.upload(buf.as_slice())?;
            let b: Box<[ffi::vxg_buffer]> = vec![ffi::vxg_buffer { ptr: p, len: buf.len() as u64 }].into_boxed_slice();
            n.buffers = b.as_ptr();
            n.n_buffers = 1;
            self.buffers.push(b);
        }
        if !children.is_empty() {
            let kids = children
                .iter()
                .map(|c| self.node(c))
                .collect::<VortexResult<Vec<_>>>()?
                .into_boxed_slice();
            n.children = kids.as_ptr();
            n.n_children = kids.len() as u32;
            self.nodes.push(kids); // the boxed slice's heap address is stable
        }
        Ok(n)
    }
}

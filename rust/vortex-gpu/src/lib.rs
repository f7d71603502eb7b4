//! `vortex-gpu`: `Array::into_canonical` on an AMD Instinct MI355X (gfx950).
//!
//! This crate is the reference-side half of the drop-in boundary declared in
//! `include/vortex_gpu.h` (the other half is `libvortex_gpu.so`, built by `vortex_amd/csrc`).
//! It registers GPU versions of the reference's encodings by their ids, so that
//!
//! ```ignore
//! let ctx = Arc::new(vortex_gpu::gpu_context());   // Context::default().with_encodings(...)
//! // ... read arrays with `ctx` (vortex-serde) or build them; then
//! let canonical = array.into_canonical()?;          // decoded on the GPU
//! ```
//!
//! decodes through the engine: `Array::into_canonical` dispatches to
//! `ArrayEncoding::canonicalize` (vortex-array/src/canonical.rs:353-357,
//! encoding/mod.rs:49-61), and the registered [`GpuEncoding`] flattens the array tree into
//! `vxg_array` descriptors (device copies of its buffers, its flexbuffer metadata converted to
//! `vxg_meta`) and calls `vxg_canonicalize`.  The outputs come back into pinned host memory and
//! are handed to Vortex as zero-copy Arrow buffers (`Buffer::from_custom_allocation`).
//!
//! A whole-file scan (the reference's `LayoutBatchStream` + `struct_to_arrow`) goes through
//! [`scan_file`]: the engine's own file reader, one H2D copy per column range, and ONE plan
//! (HIP graph) canonicalizing every column, instead of per-chunk, per-buffer calls.
//!
//! There is no CPU fallback: without a GPU the registered encodings return an error.
//!
//! UNTESTED: the build image of this project has no Rust toolchain.  `src/ffi.rs` is generated
//! from the C headers by `tools/gen_ffi_rs.py`; the Python binding (`vortex_amd/_lib.py`) that
//! the project's tests exercise follows the same calls.

mod canonical;
mod encodings;
pub mod ffi;
mod flatten;
mod meta;
mod scan;

use std::ffi::CStr;
use std::ptr;
use std::sync::OnceLock;

pub use encodings::{gpu_context, gpu_encodings, GpuEncoding};
pub use scan::{scan_file, ColumnInfo, GpuFile};
use vortex::{Array, Canonical};
use vortex_error::{vortex_bail, vortex_err, VortexResult};

/// One engine context (`vxg_ctx`) on one device.  The engine's entry points are thread-safe, so
/// a session is shared by every thread (one context per device).
pub struct GpuSession {
    ctx: *mut ffi::vxg_ctx,
    device: i32,
}

// SAFETY: vxg_ctx is internally synchronised (include/vortex_gpu.h "Threading").
unsafe impl Send for GpuSession {}
unsafe impl Sync for GpuSession {}

impl GpuSession {
    /// Open the engine on `device` after checking the library's ABI version.
    pub fn open(device: i32) -> VortexResult<Self> {
        let abi = unsafe { ffi::vxg_abi_version() };
        if abi != ffi::VXG_ABI_VERSION {
            vortex_bail!(InvalidArgument: "libvortex_gpu ABI {} but this crate was generated for {}", abi, ffi::VXG_ABI_VERSION);
        }
        let mut ctx = ptr::null_mut();
        check(unsafe { ffi::vxg_open(device, &mut ctx) })?;
        Ok(Self { ctx, device })
    }

    /// The process-wide session used by the registered encodings: device `$VORTEX_GPU_DEVICE`
    /// (default 0), opened on first use.
    pub fn global() -> VortexResult<&'static GpuSession> {
        static SESSION: OnceLock<Result<GpuSession, String>> = OnceLock::new();
        SESSION
            .get_or_init(|| {
                let device = std::env::var("VORTEX_GPU_DEVICE")
                    .ok()
                    .and_then(|d| d.parse().ok())
                    .unwrap_or(0);
                GpuSession::open(device).map_err(|e| e.to_string())
            })
            .as_ref()
            .map_err(|e| vortex_err!(ComputeError: "vortex-gpu is unavailable: {}", e))
    }

    pub fn device(&self) -> i32 {
        self.device
    }

    /// `Array::into_canonical` of `array` on the GPU (the whole tree in one engine call).
    pub fn canonicalize(&self, array: &Array) -> VortexResult<Canonical> {
        canonical::canonicalize(self, array)
    }

    pub(crate) fn raw(&self) -> *mut ffi::vxg_ctx {
        self.ctx
    }
}

impl Drop for GpuSession {
    fn drop(&mut self) {
        unsafe {
            ffi::vxg_close(self.ctx);
        }
    }
}

/// vxg_status -> VortexError (vortex-error/src/lib.rs:48-110), with the engine's message.
pub(crate) fn check(status: ffi::vxg_status) -> VortexResult<()> {
    if status == ffi::VXG_OK {
        return Ok(());
    }
    let msg = unsafe {
        let p = ffi::vxg_last_error();
        if p.is_null() {
            String::new()
        } else {
            CStr::from_ptr(p).to_string_lossy().into_owned()
        }
    };
    Err(match status {
        // the engine reports the failing index in the message, not as (idx, start, stop)
        ffi::VXG_ERR_OUT_OF_BOUNDS => vortex_err!(InvalidArgument: "out of bounds: {}", msg),
        ffi::VXG_ERR_COMPUTE => vortex_err!(ComputeError: "{}", msg),
        ffi::VXG_ERR_INVALID_ARGUMENT => vortex_err!(InvalidArgument: "{}", msg),
        ffi::VXG_ERR_INVALID_SERDE => vortex_err!(InvalidSerde: "{}", msg),
        ffi::VXG_ERR_NOT_IMPLEMENTED => vortex_err!(NotImplemented: msg, "vortex-gpu"),
        ffi::VXG_ERR_MISMATCHED_TYPES => vortex_err!(MismatchedTypes: "the engine's input types", msg),
        ffi::VXG_ERR_ASSERTION_FAILED => vortex_err!(AssertionFailed: "{}", msg),
        _ => vortex_err!(ComputeError: "HIP: {}", msg),
    })
}

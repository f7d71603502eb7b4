//! GPU registrations of the reference's encodings (vortex-array/src/implementation.rs:31-164,
//! context.rs:16-33).
//!
//! A [`GpuEncoding`] carries the reference encoding it stands in for: the same `EncodingId`
//! (name and u16 code, encoding/mod.rs:106-147), the same `with_dyn` (so typed accessors,
//! compute functions and statistics keep working unchanged), and a `canonicalize` that runs on
//! the GPU.  `gpu_context()` is `Context::default()` with these registered over the defaults by
//! code, which is all a reader (vortex-serde) or a caller needs to route decodes to the engine.
//!
//! The canonical encodings themselves (Primitive, Bool, VarBinView, Struct, Extension, Null) are
//! not wrapped: their canonicalize is the identity.  A GPU-registered encoding whose dtype the
//! engine does not produce (Struct, List or Extension chunks: no bytes are decoded there, the
//! reference only rearranges children, chunked/canonical.rs:18-120) keeps the reference's path.

use vortex::encoding::{ArrayEncoding, EncodingId, EncodingRef};
use vortex::{Array, ArrayDType, ArrayTrait, Canonical, Context};
use vortex_dtype::DType;
use vortex_error::VortexResult;

use crate::GpuSession;

#[derive(Debug)]
pub struct GpuEncoding {
    inner: EncodingRef,
}

impl GpuEncoding {
    pub const fn new(inner: EncodingRef) -> Self {
        Self { inner }
    }

    pub fn inner(&self) -> EncodingRef {
        self.inner
    }
}

impl ArrayEncoding for GpuEncoding {
    fn id(&self) -> EncodingId {
        self.inner.id()
    }

    fn canonicalize(&self, array: Array) -> VortexResult<Canonical> {
        match array.dtype() {
            DType::Struct(..) | DType::List(..) | DType::Extension(..) => self.inner.canonicalize(array),
            _ => GpuSession::global()?.canonicalize(&array),
        }
    }

    fn with_dyn(
        &self,
        array: &Array,
        f: &mut dyn for<'b> FnMut(&'b (dyn ArrayTrait + 'b)) -> VortexResult<()>,
    ) -> VortexResult<()> {
        self.inner.with_dyn(array, f)
    }
}

macro_rules! gpu_encodings {
    ($($name:ident => $inner:expr),* $(,)?) => {
        $(pub static $name: GpuEncoding = GpuEncoding::new(&$inner);)*

        /// Every GPU registration, to pass to `Context::with_encodings`.
        pub fn gpu_encodings() -> Vec<EncodingRef> {
            vec![$(&$name as EncodingRef),*]
        }
    };
}

gpu_encodings! {
    GPU_BITPACKED => vortex_fastlanes::BitPackedEncoding,
    GPU_FOR => vortex_fastlanes::FoREncoding,
    GPU_DELTA => vortex_fastlanes::DeltaEncoding,
    GPU_ALP => vortex_alp::ALPEncoding,
    GPU_ALPRD => vortex_alp::ALPRDEncoding,
    GPU_DICT => vortex_dict::DictEncoding,
    GPU_FSST => vortex_fsst::FSSTEncoding,
    GPU_RUNEND => vortex_runend::RunEndEncoding,
    GPU_RUNEND_BOOL => vortex_runend_bool::RunEndBoolEncoding,
    GPU_ZIGZAG => vortex_zigzag::ZigZagEncoding,
    GPU_BYTEBOOL => vortex_bytebool::ByteBoolEncoding,
    GPU_ROARING_BOOL => vortex_roaring::RoaringBoolEncoding,
    GPU_SPARSE => vortex::array::SparseEncoding,
    GPU_CONSTANT => vortex::array::ConstantEncoding,
    GPU_CHUNKED => vortex::array::ChunkedEncoding,
    GPU_VARBIN => vortex::array::VarBinEncoding,
}

/// `Context::default()` (context.rs:36-56) plus the GPU registrations, replacing by code.
pub fn gpu_context() -> Context {
    Context::default().with_encodings(gpu_encodings())
}

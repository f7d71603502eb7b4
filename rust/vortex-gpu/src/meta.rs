//! Flexbuffer array metadata -> `vxg_meta` (include/vortex_gpu.h), per encoding.
//!
//! Every reference encoding serialises its metadata struct with serde into a flexbuffer map
//! (vortex-array/src/metadata.rs:35-47); this module reads those maps by field name, exactly the
//! fields the engine needs, with the serde conventions of the reference's types:
//! `ValidityMetadata` (validity.rs:24-30) and other unit enums are strings, `PType`
//! (vortex-dtype/src/ptype.rs:17-32) is a lower-case string, `Nullability` a bool, a
//! `ScalarValue` its primitive value (or null).  Unit metadata structs (ZigZag, RoaringBool)
//! serialise to null.  The C++ twin of this module is the file reader (vortex_amd/csrc/serde.cpp).

use flexbuffers::{FlexBufferType, MapReader, Reader};
use vortex_dtype::{DType, PType};
use vortex_error::{vortex_bail, vortex_err, VortexResult};

use crate::ffi;

pub(crate) fn ptype_code(p: PType) -> u8 {
    match p {
        PType::U8 => 0,
        PType::U16 => 1,
        PType::U32 => 2,
        PType::U64 => 3,
        PType::I8 => 4,
        PType::I16 => 5,
        PType::I32 => 6,
        PType::I64 => 7,
        PType::F16 => 8,
        PType::F32 => 9,
        PType::F64 => 10,
    }
}

/// Inverse of [`ptype_code`] (the reader's column ptypes).
pub(crate) fn ptype_of_code(c: u8) -> VortexResult<PType> {
    Ok(match c {
        0 => PType::U8,
        1 => PType::U16,
        2 => PType::U32,
        3 => PType::U64,
        4 => PType::I8,
        5 => PType::I16,
        6 => PType::I32,
        7 => PType::I64,
        8 => PType::F16,
        9 => PType::F32,
        10 => PType::F64,
        _ => vortex_bail!(InvalidSerde: "unknown ptype code {}", c),
    })
}

fn ptype_width(p: PType) -> usize {
    match p {
        PType::U8 | PType::I8 => 1,
        PType::U16 | PType::I16 | PType::F16 => 2,
        PType::U32 | PType::I32 | PType::F32 => 4,
        PType::U64 | PType::I64 | PType::F64 => 8,
    }
}

fn ptype_from_name(s: &str) -> VortexResult<u8> {
    Ok(match s {
        "u8" => 0,
        "u16" => 1,
        "u32" => 2,
        "u64" => 3,
        "i8" => 4,
        "i16" => 5,
        "i32" => 6,
        "i64" => 7,
        "f16" => 8,
        "f32" => 9,
        "f64" => 10,
        _ => vortex_bail!(InvalidSerde: "unknown ptype {:?}", s),
    })
}

fn validity_code(s: &str) -> VortexResult<u8> {
    Ok(match s {
        "NonNullable" => ffi::VXG_VALIDITY_NON_NULLABLE as u8,
        "AllValid" => ffi::VXG_VALIDITY_ALL_VALID as u8,
        "AllInvalid" => ffi::VXG_VALIDITY_ALL_INVALID as u8,
        "Array" => ffi::VXG_VALIDITY_ARRAY as u8,
        _ => vortex_bail!(InvalidSerde: "unknown validity {:?}", s),
    })
}

struct Map<'a>(MapReader<&'a [u8]>);

impl<'a> Map<'a> {
    fn get(&self, key: &str) -> VortexResult<Reader<&'a [u8]>> {
        self.0
            .index(key)
            .map_err(|e| vortex_err!(InvalidSerde: "metadata field {}: {}", key, e))
    }
    fn u64(&self, key: &str) -> VortexResult<u64> {
        Ok(self.get(key)?.as_u64())
    }
    fn bool(&self, key: &str) -> VortexResult<bool> {
        Ok(self.get(key)?.as_bool())
    }
    fn string(&self, key: &str) -> VortexResult<String> {
        Ok(self.get(key)?.as_str().to_string())
    }
    fn ptype(&self, key: &str) -> VortexResult<u8> {
        ptype_from_name(&self.string(key)?)
    }
    fn validity(&self) -> VortexResult<u8> {
        validity_code(&self.string("validity")?)
    }
}

fn map<'a>(bytes: Option<&'a [u8]>, what: &str) -> VortexResult<Map<'a>> {
    let bytes = bytes.ok_or_else(|| vortex_err!(InvalidSerde: "{} requires metadata bytes", what))?;
    let root = Reader::get_root(bytes).map_err(|e| vortex_err!(InvalidSerde: "{} metadata: {}", what, e))?;
    Ok(Map(root
        .get_map()
        .map_err(|e| vortex_err!(InvalidSerde: "{} metadata is not a map: {}", what, e))?))
}

/// A ScalarValue (FoR reference, Sparse fill, Constant) as the little-endian bytes of `dtype`
/// -> (is_null, bytes).
fn scalar_bytes(r: &Reader<&[u8]>, dtype: &DType) -> VortexResult<(bool, [u8; 16])> {
    let mut out = [0u8; 16];
    if r.flexbuffer_type() == FlexBufferType::Null {
        return Ok((true, out));
    }
    match dtype {
        DType::Bool(_) => out[0] = r.as_bool() as u8,
        DType::Primitive(p, _) => {
            let w = ptype_width(*p);
            let bytes: [u8; 8] = match p {
                PType::F32 => (u64::from((r.as_f64() as f32).to_bits())).to_le_bytes(),
                PType::F64 => r.as_f64().to_bits().to_le_bytes(),
                PType::F16 => (vortex_dtype::half::f16::from_f64(r.as_f64()).to_bits() as u64).to_le_bytes(),
                PType::I8 | PType::I16 | PType::I32 | PType::I64 => r.as_i64().to_le_bytes(),
                _ => r.as_u64().to_le_bytes(),
            };
            out[..w].copy_from_slice(&bytes[..w]);
        }
        _ => vortex_bail!(NotImplemented: "scalar of this dtype", "vortex-gpu"),
    }
    Ok((false, out))
}

/// (vxg_meta, ValidityMetadata code) of one array node.  `nchildren` decides the optional
/// children the metadata does not name (ALP patches).
pub(crate) fn convert(
    code: u16,
    dtype: &DType,
    bytes: Option<&[u8]>,
    nchildren: usize,
) -> VortexResult<(ffi::vxg_meta, u8)> {
    let mut m: ffi::vxg_meta = unsafe { std::mem::zeroed() };
    let mut validity = ffi::VXG_VALIDITY_NON_NULLABLE as u8;
    let c = code as i32;
    // union field stores (nested places need `unsafe`)
    #[allow(unused_unsafe)]
    unsafe {
        match c {
            ffi::VXG_ENC_PRIMITIVE | ffi::VXG_ENC_BYTE_BOOL => {
                validity = map(bytes, "Primitive")?.validity()?;
            }
            ffi::VXG_ENC_BOOL => {
                let mm = map(bytes, "Bool")?;
                validity = mm.validity()?;
                m.boolean.first_byte_bit_offset = mm.u64("first_byte_bit_offset")? as u8;
            }
            ffi::VXG_ENC_VARBIN => {
                let mm = map(bytes, "VarBin")?;
                validity = mm.validity()?;
                m.varbin.offsets_ptype = mm.ptype("offsets_ptype")?;
                m.varbin.bytes_len = mm.u64("bytes_len")?;
            }
            ffi::VXG_ENC_VARBINVIEW => {
                let mm = map(bytes, "VarBinView")?;
                validity = mm.validity()?;
                m.varbinview.n_buffers = mm.get("buffer_lens")?.as_vector().len() as u32;
            }
            ffi::VXG_ENC_SPARSE => {
                let mm = map(bytes, "Sparse")?;
                m.sparse.indices_offset = mm.u64("indices_offset")?;
                m.sparse.indices_len = mm.u64("indices_len")?;
                let (null, b) = scalar_bytes(&mm.get("fill_value")?, dtype)?;
                m.sparse.fill_is_null = null as u8;
                m.sparse.fill = b;
            }
            ffi::VXG_ENC_CONSTANT => {
                let mm = map(bytes, "Constant")?;
                let (null, b) = scalar_bytes(&mm.get("scalar_value")?, dtype)?;
                m.constant.is_null = null as u8;
                m.constant.scalar = b;
            }
            ffi::VXG_ENC_CHUNKED => {
                m.chunked.nchunks = map(bytes, "Chunked")?.u64("nchunks")?;
            }
            ffi::VXG_ENC_ALP => {
                let mm = map(bytes, "ALP")?;
                let ex = mm.get("exponents")?.get_map().map_err(|e| vortex_err!(InvalidSerde: "{}", e))?;
                m.alp.e = ex.index("e").map_err(|e| vortex_err!(InvalidSerde: "{}", e))?.as_u8();
                m.alp.f = ex.index("f").map_err(|e| vortex_err!(InvalidSerde: "{}", e))?.as_u8();
                m.alp.has_patches = (nchildren > 1) as u8;
            }
            ffi::VXG_ENC_ALP_RD => {
                let mm = map(bytes, "ALPRD")?;
                m.alprd.right_bit_width = mm.u64("right_bit_width")? as u8;
                m.alprd.dict_len = mm.u64("dict_len")? as u8;
                m.alprd.left_parts_ptype = mm.ptype("left_parts_ptype")?;
                m.alprd.has_exceptions = mm.bool("has_exceptions")? as u8;
                let d = mm.get("dict")?.as_vector();
                for i in 0..d.len().min(8) {
                    m.alprd.dict[i] = d.idx(i).as_u16();
                }
            }
            ffi::VXG_ENC_DICT => {
                let mm = map(bytes, "Dict")?;
                m.dict.codes_ptype = mm.ptype("codes_ptype")?;
                m.dict.values_len = mm.u64("values_len")?;
            }
            ffi::VXG_ENC_FL_BITPACKED => {
                let mm = map(bytes, "BitPacked")?;
                validity = mm.validity()?;
                m.bitpacked.bit_width = mm.u64("bit_width")? as u8;
                m.bitpacked.offset = mm.u64("offset")? as u16;
                m.bitpacked.has_patches = mm.bool("has_patches")? as u8;
            }
            ffi::VXG_ENC_FL_DELTA => {
                let mm = map(bytes, "Delta")?;
                validity = mm.validity()?;
                m.delta.deltas_len = mm.u64("deltas_len")?;
                m.delta.offset = mm.u64("offset")? as u16;
            }
            ffi::VXG_ENC_FL_FOR => {
                let mm = map(bytes, "FoR")?;
                let (_, b) = scalar_bytes(&mm.get("reference")?, dtype)?;
                m.for_.reference = u64::from_le_bytes(b[..8].try_into().unwrap_or([0; 8]));
                m.for_.shift = mm.u64("shift")? as u8;
            }
            ffi::VXG_ENC_FSST => {
                let mm = map(bytes, "FSST")?;
                m.fsst.symbols_len = mm.u64("symbols_len")?;
                m.fsst.codes_nullable = mm.bool("codes_nullability")? as u8;
                m.fsst.uncompressed_lengths_ptype = mm.ptype("uncompressed_lengths_ptype")?;
            }
            ffi::VXG_ENC_RUN_END => {
                let mm = map(bytes, "RunEnd")?;
                validity = mm.validity()?;
                m.runend.ends_ptype = mm.ptype("ends_ptype")?;
                m.runend.num_runs = mm.u64("num_runs")?;
                m.runend.offset = mm.u64("offset")?;
            }
            ffi::VXG_ENC_RUN_END_BOOL => {
                let mm = map(bytes, "RunEndBool")?;
                validity = mm.validity()?;
                m.runendbool.start = mm.bool("start")? as u8;
                m.runendbool.ends_ptype = mm.ptype("ends_ptype")?;
                m.runendbool.num_runs = mm.u64("num_runs")?;
                m.runendbool.offset = mm.u64("offset")?;
            }
            ffi::VXG_ENC_ZIGZAG | ffi::VXG_ENC_ROARING_BOOL => {}
            _ => vortex_bail!(NotImplemented: format!("GPU canonicalize of encoding {}", code), "vortex-gpu"),
        }
    }
    Ok((m, validity))
}

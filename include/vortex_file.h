/*
 * vortex_file.h — C ABI of the Vortex file reader that feeds the MI355X decode engine.
 *
 * A Vortex file (vortex-serde LayoutWriter output, vortex-serde/src/layouts/write/writer.rs:
 * 40-201) is parsed on the host, straight from its bytes: EOF (version u16 + "VRTX", layouts/
 * mod.rs:8-12), the 32-byte Postscript, the Schema message and the Footer flatbuffer (footer.fbs,
 * read/footer.rs:140-187), the Column -> Chunked -> Flat layout tree (read/layouts/{column,chunked,flat}.rs), each
 * column's row_offset metadata table, and every chunk's IPC Batch message (message.fbs;
 * ArrayBufferReader::read, message_reader.rs:249-306): its flatbuffer `Array` tree (array.fbs)
 * with the per-encoding flexbuffer metadata (metadata.rs:35-47) and its 64-byte-aligned buffers
 * (lib.rs:15).  The result is the `vxg_array` tree `ArrayView::try_new` (vortex-array/src/
 * view.rs:45-83) would resolve: encodings by their u16 id, each child's dtype and length derived
 * exactly as the owning encoding's accessors derive them, buffers pointing into the caller's
 * copy of the file bytes.  No flatbuffers/flexbuffers library is used (none in this image):
 * both formats are decoded by hand with bounds checks (malformed input -> VXG_ERR_INVALID_SERDE).
 *
 * Intended use ("file bytes in, Arrow buffers out"): keep the file in pinned host memory, copy
 * the byte range of the chunks to decode to HBM with ONE copy per column range (the messages of
 * a column are contiguous), call vxg_file_column_array with that device region, and hand the
 * tree to vxg_canonicalize / vxg_plan_create (include/vortex_gpu.h).
 */
#ifndef VORTEX_FILE_H
#define VORTEX_FILE_H

#include <stddef.h>
#include <stdint.h>

#include "vortex_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vxg_file vxg_file;

/* One top-level column (a field of the file's Struct schema). */
typedef struct vxg_file_column {
    const char* name;               /* field name, NUL-terminated (owned by the file) */
    uint8_t dtype;                  /* VXG_DTYPE_* (Extension columns: of the storage dtype) */
    uint8_t ptype;                  /* VXG_* ptype for primitive (storage) dtypes */
    uint8_t nullable;
    uint8_t is_extension;           /* DType::Extension: chunks are ExtensionArray(storage) */
    uint32_t n_chunks;
    const char* extension_id;       /* e.g. "vortex.date", or NULL */
    const uint8_t* extension_metadata;
    uint64_t extension_metadata_len;
    uint64_t rows;
} vxg_file_column;

/* One chunk (one IPC Batch message, a FlatLayout) of a column. */
typedef struct vxg_file_chunk {
    uint64_t row_offset;     /* first row (the column's row_offset metadata table) */
    uint64_t rows;           /* Batch.length */
    uint64_t message_begin;  /* file byte range of the message (FlatLayout buffer) */
    uint64_t message_end;
    uint64_t buffers_begin;  /* first byte of the message's buffers (64-byte aligned) */
} vxg_file_chunk;

/* Parse a Vortex file held in host memory.  `bytes` must stay valid (and unchanged) until
 * vxg_file_close: chunk messages are parsed from it lazily.  Read/footer.rs:140-187 checks. */
vxg_status vxg_file_open(const void* bytes, uint64_t len, vxg_file** out);
vxg_status vxg_file_close(vxg_file* file);
vxg_status vxg_file_info(const vxg_file* file, uint64_t* row_count, uint32_t* n_columns);
vxg_status vxg_file_column_info(const vxg_file* file, uint32_t column, vxg_file_column* out);
vxg_status vxg_file_chunk_info(const vxg_file* file, uint32_t column, uint32_t chunk, vxg_file_chunk* out);

/* Chunk offsets of chunks [chunk_begin, chunk_end) of a column relative to the first one
 * (chunk_end - chunk_begin + 1 u64 values into host_out): the chunk_offsets child of the
 * ChunkedArray the reader builds (array/chunked/mod.rs:54-70). */
vxg_status vxg_file_chunk_offsets(const vxg_file* file, uint32_t column, uint32_t chunk_begin,
                                  uint32_t chunk_end, uint64_t* host_out);

/* The array tree of chunks [chunk_begin, chunk_end) of a column: a ChunkedArray (encoding
 * VXG_ENC_CHUNKED, children = [chunk_offsets, chunk...]) whose chunks are the messages' arrays
 * (an Extension column's chunks are their storage arrays).  Every buffer pointer is
 * `region + (file offset of the buffer - region_file_offset)`: `region` is the caller's copy
 * (e.g. in HBM) of file bytes [region_file_offset, region_file_offset + region_len), which must
 * cover the chunks' messages (else InvalidArgument).  region = NULL, region_file_offset = 0
 * gives pointers equal to file offsets (inspection without a device).  chunk_offsets_dev: a
 * device copy of vxg_file_chunk_offsets (or NULL; the engine does not read it).  The tree is
 * owned by the file and stays valid until vxg_file_close. */
vxg_status vxg_file_column_array(vxg_file* file, uint32_t column, uint32_t chunk_begin, uint32_t chunk_end,
                                 const void* region, uint64_t region_file_offset, uint64_t region_len,
                                 const void* chunk_offsets_dev, const vxg_array** out);

#ifdef __cplusplus
}
#endif
#endif /* VORTEX_FILE_H */

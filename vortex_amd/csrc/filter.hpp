// filter.hpp — compute::filter kernels (filter.hip); internal, not the C ABI.
#pragma once

#include "vxg_internal.hpp"

namespace vxg {

// Rows per filter tile: one wavefront owns 64 predicate words of 64 rows.
constexpr uint64_t kFilterTileRows = 4096;

inline uint64_t filter_tiles(uint64_t n) { return (n + kFilterTileRows - 1) / kFilterTileRows; }

// Predicate = LSB bit buffer read as u64 words (the caller pads it to whole words, bits past
// len zero).  tile_off: filter_tiles(n) + 1 u64; tile_off[tiles] = true_count after the scan.
vxg_status launch_filter_count(const uint64_t* mask, uint64_t n, uint64_t* tile_off, hipStream_t s);

// Compact `width`-byte values (1,2,4,8,16) of the selected rows into out (tile_off scanned).
vxg_status launch_filter_values(const uint64_t* mask, uint64_t n, const uint64_t* tile_off, const void* in,
                                int width, void* out, hipStream_t s);

// Compact the bits of an LSB bit buffer (src, bit 0 = row 0) of the selected rows into the
// zeroed bit buffer dst (u32 words).
vxg_status launch_filter_bits(const uint64_t* mask, uint64_t n, const uint64_t* tile_off, const uint8_t* src,
                              void* dst, hipStream_t s);

// Strings: views (already compacted, n rows; valid = their LSB validity or null; null rows get
// zero views and no bytes) -> per-tile byte totals for a new heap.
// heap_off: filter_tiles(n) + 1 u64, scanned in place; heap_off[tiles] = heap bytes.
vxg_status launch_view_heap_sizes(const uint8_t* views, uint64_t n, const uint8_t* valid, uint64_t* heap_off,
                                  hipStream_t s);
// Rewrite the views over the new heap (one buffer, index 0) and copy each string's bytes
// (inline ones from the view itself, others from buffers[buffer_index] + offset).
vxg_status launch_view_heap_build(uint8_t* views, uint64_t n, const uint8_t* valid, const uint64_t* heap_off,
                                  const uint8_t* const* bufs,
                                  uint32_t n_bufs, uint8_t* heap, uint32_t* err, hipStream_t s);

}  // namespace vxg

// Page directory of one Parquet column chunk: the Thrift-compact PageHeader of every page (reference
// reader: src/data/readers/parquet_reader.rs reads the `text` column through the `parquet` crate;
// here the text column can be decoded on the GPU, csrc/hip/parquet.hip, from this directory).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace tb {

enum PqPageType : int32_t { PQ_DATA_PAGE = 0, PQ_INDEX_PAGE = 1, PQ_DICTIONARY_PAGE = 2, PQ_DATA_PAGE_V2 = 3 };

struct PqPageInfo {
  int32_t type = -1;
  int64_t data_off = 0;          // first byte after the header, relative to the chunk
  int32_t compressed_size = 0;
  int32_t uncompressed_size = 0;
  int32_t num_values = 0;        // data pages: values incl. nulls; dictionary: entries
  int32_t encoding = 0;          // values encoding (0 PLAIN, 2 PLAIN_DICTIONARY, 8 RLE_DICTIONARY)
  int32_t def_encoding = 3;      // v1: definition-level encoding (3 RLE)
  int32_t num_nulls = 0;         // v2
  int32_t def_len = 0;           // v2: definition-level bytes (stored uncompressed)
  int32_t rep_len = 0;           // v2: repetition-level bytes (stored uncompressed)
  int32_t v2_compressed = 1;     // v2: is_compressed
};

// Pages of the chunk bytes [0, n). Throws std::runtime_error on a malformed header.
std::vector<PqPageInfo> parquet_pages(const uint8_t* buf, size_t n);

}  // namespace tb

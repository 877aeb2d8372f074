// Thrift compact-protocol reader for Parquet PageHeader structs (parquet.thrift: PageHeader,
// DataPageHeader, DictionaryPageHeader, DataPageHeaderV2). Only the fields the GPU decoder needs
// are kept; everything else (statistics, CRC, index pages) is skipped structurally.
#include "parquet_pages.h"

#include <stdexcept>
#include <string>

namespace tb {
namespace {

enum : int { T_STOP = 0, T_TRUE = 1, T_FALSE = 2, T_BYTE = 3, T_I16 = 4, T_I32 = 5, T_I64 = 6, T_DOUBLE = 7,
             T_BINARY = 8, T_LIST = 9, T_SET = 10, T_MAP = 11, T_STRUCT = 12 };

struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  [[noreturn]] void fail(const char* what) const { throw std::runtime_error(std::string("parquet page header: ") + what); }
  uint8_t byte() {
    if (p >= e) fail("truncated");
    return *p++;
  }
  uint64_t varint() {
    uint64_t v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      const uint8_t b = byte();
      v |= (uint64_t)(b & 0x7F) << shift;
      if (!(b & 0x80)) return v;
    }
    fail("varint too long");
  }
  int64_t zigzag() {
    const uint64_t v = varint();
    return (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
  }
  void skip_bytes(uint64_t n) {
    if ((uint64_t)(e - p) < n) fail("truncated");
    p += n;
  }
  void skip(int type, int depth = 0) {
    if (depth > 32) fail("nesting too deep");
    switch (type) {
      case T_TRUE: case T_FALSE: return;  // value in the type nibble (struct field) or one byte (list)
      case T_BYTE: byte(); return;
      case T_I16: case T_I32: case T_I64: varint(); return;
      case T_DOUBLE: skip_bytes(8); return;
      case T_BINARY: skip_bytes(varint()); return;
      case T_LIST: case T_SET: {
        const uint8_t h = byte();
        uint64_t n = h >> 4;
        const int et = h & 0x0F;
        if (n == 15) n = varint();
        for (uint64_t i = 0; i < n; ++i) {
          if (et == T_TRUE || et == T_FALSE) byte();
          else skip(et, depth + 1);
        }
        return;
      }
      case T_MAP: {
        const uint64_t n = varint();
        if (!n) return;
        const uint8_t kv = byte();
        for (uint64_t i = 0; i < n; ++i) {
          skip(kv >> 4, depth + 1);
          skip(kv & 0x0F, depth + 1);
        }
        return;
      }
      case T_STRUCT: struct_fields([&](int, int t) { skip(t, depth + 1); }); return;
      default: fail("unknown field type");
    }
  }
  // Calls f(field id, type) for every field of a struct until STOP; f must consume the value.
  template <class F>
  void struct_fields(F&& f) {
    int last = 0;
    for (;;) {
      const uint8_t h = byte();
      const int type = h & 0x0F;
      if (type == T_STOP) return;
      const int delta = h >> 4;
      const int id = delta ? last + delta : (int)zigzag();
      last = id;
      f(id, type);
    }
  }
  int32_t i32(int type) {
    if (type != T_I32) fail("expected i32");
    return (int32_t)zigzag();
  }
};

}  // namespace

std::vector<PqPageInfo> parquet_pages(const uint8_t* buf, size_t n) {
  std::vector<PqPageInfo> out;
  size_t pos = 0;
  while (pos < n) {
    Reader r{buf + pos, buf + n};
    PqPageInfo pg;
    r.struct_fields([&](int id, int type) {
      switch (id) {
        case 1: pg.type = r.i32(type); break;
        case 2: pg.uncompressed_size = r.i32(type); break;
        case 3: pg.compressed_size = r.i32(type); break;
        case 5:  // DataPageHeader
          if (type != T_STRUCT) r.fail("data_page_header");
          r.struct_fields([&](int fid, int ft) {
            if (fid == 1) pg.num_values = r.i32(ft);
            else if (fid == 2) pg.encoding = r.i32(ft);
            else if (fid == 3) pg.def_encoding = r.i32(ft);
            else r.skip(ft);
          });
          break;
        case 7:  // DictionaryPageHeader
          if (type != T_STRUCT) r.fail("dictionary_page_header");
          r.struct_fields([&](int fid, int ft) {
            if (fid == 1) pg.num_values = r.i32(ft);
            else if (fid == 2) pg.encoding = r.i32(ft);
            else r.skip(ft);
          });
          break;
        case 8:  // DataPageHeaderV2
          if (type != T_STRUCT) r.fail("data_page_header_v2");
          r.struct_fields([&](int fid, int ft) {
            if (fid == 1) pg.num_values = r.i32(ft);
            else if (fid == 2) pg.num_nulls = r.i32(ft);
            else if (fid == 4) pg.encoding = r.i32(ft);
            else if (fid == 5) pg.def_len = r.i32(ft);
            else if (fid == 6) pg.rep_len = r.i32(ft);
            else if (fid == 7) pg.v2_compressed = ft == T_TRUE ? 1 : 0;  // bool: value in the type nibble
            else r.skip(ft);
          });
          break;
        default:
          r.skip(type);
      }
    });
    if (pg.type < 0 || pg.compressed_size < 0 || pg.uncompressed_size < 0 || pg.num_values < 0)
      throw std::runtime_error("parquet page header: missing or negative field");
    pg.data_off = (int64_t)(r.p - buf);
    if ((uint64_t)pg.data_off + (uint64_t)pg.compressed_size > n)
      throw std::runtime_error("parquet page header: page runs past the column chunk");
    pos = (size_t)pg.data_off + (size_t)pg.compressed_size;
    out.push_back(pg);
  }
  return out;
}

}  // namespace tb

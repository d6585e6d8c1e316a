// Implementation of tf_formats.h (see header for scope).
#include "tf_formats.h"

#include <nmmintrin.h>
#include <zlib.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <tuple>

namespace dtfe_rt {

// ================================================================= crc32c
static uint32_t g_table[8][256];
static bool g_table_init = false;
static bool g_hw = false;

static void crc_init() {
  if (g_table_init) return;
  const uint32_t poly = 0x82f63b78u;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : (c >> 1);
    g_table[0][i] = c;
  }
  for (int t = 1; t < 8; ++t)
    for (uint32_t i = 0; i < 256; ++i) g_table[t][i] = (g_table[t - 1][i] >> 8) ^ g_table[0][g_table[t - 1][i] & 0xff];
  __builtin_cpu_init();
  g_hw = __builtin_cpu_supports("sse4.2");
  g_table_init = true;
}

__attribute__((target("sse4.2"))) static uint32_t crc_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32;
}

uint32_t crc32c_extend(uint32_t init, const void* data, size_t n) {
  crc_init();
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t crc = init ^ 0xffffffffu;
  if (g_hw) {
    crc = crc_hw(crc, p, n);
  } else {
    while (n--) crc = (crc >> 8) ^ g_table[0][(crc ^ *p++) & 0xff];
  }
  return crc ^ 0xffffffffu;
}

// ================================================================= encoding
void put_fixed32(std::string& s, uint32_t v) {
  char b[4];
  std::memcpy(b, &v, 4);
  s.append(b, 4);
}
void put_fixed64(std::string& s, uint64_t v) {
  char b[8];
  std::memcpy(b, &v, 8);
  s.append(b, 8);
}
void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)(v | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}
bool get_varint(const char*& p, const char* end, uint64_t& v) {
  v = 0;
  for (int shift = 0; shift <= 63 && p < end; shift += 7) {
    const uint8_t b = (uint8_t)*p++;
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) return true;
  }
  return false;
}
uint32_t get_fixed32(const char* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
uint64_t get_fixed64(const char* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}

void PbWriter::varint(uint64_t v) { put_varint(buf, v); }
void PbWriter::fixed32(int field, uint32_t v) { key(field, 5); put_fixed32(buf, v); }
void PbWriter::fixed64(int field, uint64_t v) { key(field, 1); put_fixed64(buf, v); }
void PbWriter::f32(int field, float v) { uint32_t u; std::memcpy(&u, &v, 4); fixed32(field, u); }
void PbWriter::f64(int field, double v) { uint64_t u; std::memcpy(&u, &v, 8); fixed64(field, u); }

bool pb_parse(const std::string& msg, std::vector<PbField>& out) {
  const char* p = msg.data();
  const char* end = p + msg.size();
  while (p < end) {
    uint64_t k;
    if (!get_varint(p, end, k)) return false;
    PbField f{(int)(k >> 3), (int)(k & 7), 0, {}};
    switch (f.wt) {
      case 0:
        if (!get_varint(p, end, f.v)) return false;
        break;
      case 1:
        if (end - p < 8) return false;
        f.v = get_fixed64(p);
        p += 8;
        break;
      case 5:
        if (end - p < 4) return false;
        f.v = get_fixed32(p);
        p += 4;
        break;
      case 2: {
        uint64_t n;
        if (!get_varint(p, end, n) || (uint64_t)(end - p) < n) return false;
        f.s.assign(p, n);
        p += n;
        break;
      }
      default:
        return false;
    }
    out.push_back(std::move(f));
  }
  return true;
}

// ================================================================= SSTable
namespace {
struct BlockBuilder {
  std::string buf;
  std::vector<uint32_t> restarts{0};
  std::string last_key;
  int counter = 0;
  int interval = 16;
  size_t entries = 0;

  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter < interval) {
      const size_t mn = std::min(last_key.size(), key.size());
      while (shared < mn && last_key[shared] == key[shared]) ++shared;
    } else {
      restarts.push_back((uint32_t)buf.size());
      counter = 0;
    }
    put_varint(buf, shared);
    put_varint(buf, key.size() - shared);
    put_varint(buf, value.size());
    buf.append(key.data() + shared, key.size() - shared);
    buf += value;
    last_key = key;
    ++counter;
    ++entries;
  }
  size_t size_estimate() const { return buf.size() + restarts.size() * 4 + 4; }
  std::string finish() {
    std::string out = buf;
    for (uint32_t r : restarts) put_fixed32(out, r);
    put_fixed32(out, (uint32_t)restarts.size());
    return out;
  }
};

std::string handle(uint64_t off, uint64_t size) {
  std::string s;
  put_varint(s, off);
  put_varint(s, size);
  return s;
}

void emit_block(std::string& file, const std::string& contents, uint64_t& off, uint64_t& size) {
  off = file.size();
  size = contents.size();
  file += contents;
  const char type = 0;  // kNoCompression
  uint32_t crc = crc32c(contents.data(), contents.size());
  crc = crc32c_extend(crc, &type, 1);
  file.push_back(type);
  put_fixed32(file, crc_mask(crc));
}

const uint64_t kTableMagic = 0xdb4775248b80fb57ull;

bool parse_block(const std::string& file, uint64_t off, uint64_t size,
                 std::vector<std::pair<std::string, std::string>>& out, std::string* err) {
  if (off + size + 5 > file.size()) { if (err) *err = "block out of range"; return false; }
  const char* b = file.data() + off;
  // verify trailer crc
  uint32_t crc = crc32c(b, size + 1);
  if (crc_mask(crc) != get_fixed32(b + size + 1)) { if (err) *err = "block crc mismatch"; return false; }
  if (b[size] != 0) { if (err) *err = "compressed blocks not supported"; return false; }
  if (size < 4) { if (err) *err = "short block"; return false; }
  const uint32_t nrest = get_fixed32(b + size - 4);
  const char* end = b + size - 4 - 4 * (size_t)nrest;
  const char* p = b;
  std::string key;
  while (p < end) {
    uint64_t shared, unshared, vlen;
    if (!get_varint(p, end, shared) || !get_varint(p, end, unshared) || !get_varint(p, end, vlen)) {
      if (err) *err = "bad block entry";
      return false;
    }
    if ((uint64_t)(end - p) < unshared + vlen || shared > key.size()) { if (err) *err = "bad entry size"; return false; }
    key.resize(shared);
    key.append(p, unshared);
    p += unshared;
    out.emplace_back(key, std::string(p, vlen));
    p += vlen;
  }
  return true;
}
}  // namespace

std::string sstable_build(const std::vector<std::pair<std::string, std::string>>& kv, size_t block_size) {
  std::string file;
  BlockBuilder data, index;
  std::string last_key;
  auto flush = [&]() {
    if (data.entries == 0) return;
    uint64_t off, size;
    emit_block(file, data.finish(), off, size);
    index.add(last_key, handle(off, size));  // separator = last key of the block (>= every key in it)
    data = BlockBuilder();
  };
  for (const auto& e : kv) {
    data.add(e.first, e.second);
    last_key = e.first;
    if (data.size_estimate() >= block_size) flush();
  }
  flush();
  uint64_t meta_off, meta_size, idx_off, idx_size;
  BlockBuilder meta;
  emit_block(file, meta.finish(), meta_off, meta_size);
  emit_block(file, index.finish(), idx_off, idx_size);
  std::string footer = handle(meta_off, meta_size) + handle(idx_off, idx_size);
  footer.resize(40, '\0');
  put_fixed64(footer, kTableMagic);
  file += footer;
  return file;
}

bool sstable_parse(const std::string& file, std::vector<std::pair<std::string, std::string>>& out, std::string* err) {
  if (file.size() < 48) { if (err) *err = "file too short"; return false; }
  const char* f = file.data() + file.size() - 48;
  if (get_fixed64(f + 40) != kTableMagic) { if (err) *err = "bad table magic"; return false; }
  const char* p = f;
  const char* end = f + 40;
  uint64_t mo, ms, io, is;
  if (!get_varint(p, end, mo) || !get_varint(p, end, ms) || !get_varint(p, end, io) || !get_varint(p, end, is)) {
    if (err) *err = "bad footer";
    return false;
  }
  std::vector<std::pair<std::string, std::string>> idx;
  if (!parse_block(file, io, is, idx, err)) return false;
  for (const auto& e : idx) {
    const char* q = e.second.data();
    uint64_t bo, bs;
    if (!get_varint(q, q + e.second.size(), bo) || !get_varint(q, q + e.second.size(), bs)) {
      if (err) *err = "bad block handle";
      return false;
    }
    if (!parse_block(file, bo, bs, out, err)) return false;
  }
  return true;
}

// ================================================================= bundle
static std::string encode_shape(const std::vector<int64_t>& shape) {
  PbWriter s;
  for (int64_t d : shape) {
    PbWriter dim;
    if (d) dim.i64(1, d);
    s.bytes(2, dim.buf);
  }
  return s.buf;
}

// TensorSliceProto { repeated Extent extent = 1; }  Extent { int64 start = 1; int64 length = 2 (oneof) }
// A full extent is an empty Extent (TensorSlice::AsProto).
static std::string encode_slice(const SliceSpec& sl) {
  PbWriter w;
  for (const auto& d : sl) {
    PbWriter ext;
    if (d.second != -1) {
      if (d.first) ext.i64(1, d.first);
      ext.i64(2, d.second);
    }
    w.bytes(1, ext.buf);
  }
  return w.buf;
}

std::string encode_bundle_entry(const BundleEntry& e) {
  PbWriter w;
  if (e.dtype) w.u64(1, (uint64_t)e.dtype);
  w.bytes(2, encode_shape(e.shape));
  if (e.offset) w.i64(4, e.offset);
  if (e.size) w.i64(5, e.size);
  if (e.size || e.slices.empty()) w.fixed32(6, crc_mask(e.crc));  // (a sliced tensor's entry holds no data)
  for (const auto& sl : e.slices) w.bytes(7, encode_slice(sl));
  return w.buf;
}

// ---- OrderedCode (tensorflow/core/lib/strings/ordered_code.cc), the three writers the slice key uses
static void oc_write_num_increasing(std::string& dest, uint64_t val) {
  unsigned char buf[9];
  int len = 0;
  while (val > 0) {
    ++len;
    buf[9 - len] = (unsigned char)(val & 0xff);
    val >>= 8;
  }
  buf[9 - len - 1] = (unsigned char)len;
  ++len;
  dest.append(reinterpret_cast<const char*>(buf + 9 - len), len);
}

static void oc_write_string(std::string& dest, const std::string& s) {
  for (unsigned char c : s) {  // 0x00 -> 0x00 0xff, 0xff -> 0xff 0x00
    if (c == 0x00) { dest.push_back('\x00'); dest.push_back('\xff'); }
    else if (c == 0xff) { dest.push_back('\xff'); dest.push_back('\x00'); }
    else dest.push_back((char)c);
  }
  dest.push_back('\x00');  // separator
  dest.push_back('\x01');
}

static void oc_write_signed_num_increasing(std::string& dest, int64_t val) {
  static const unsigned char kHeader[11][2] = {{0, 0},    {0x80, 0}, {0xc0, 0}, {0xe0, 0},    {0xf0, 0},   {0xf8, 0},
                                               {0xfc, 0}, {0xfe, 0}, {0xff, 0}, {0xff, 0x80}, {0xff, 0xc0}};
  const uint64_t x = val < 0 ? ~(uint64_t)val : (uint64_t)val;
  if (x < 64) {
    dest.push_back((char)(kHeader[1][0] ^ (unsigned char)val));
    return;
  }
  // bits needed (incl. sign) -> encoded length: 7 payload bits per byte minus the header's
  int bits = 64;
  while (bits > 0 && !((x >> (bits - 1)) & 1)) --bits;
  const int len = bits / 7 + 1;  // x >= 64: bits >= 7 -> len >= 2 (each byte carries 7 header/value bits)
  unsigned char buf[10];
  const unsigned char sign = val < 0 ? 0xff : 0x00;
  buf[0] = buf[1] = sign;
  for (int i = 0; i < 8; ++i) buf[2 + i] = (unsigned char)(((uint64_t)val) >> (8 * (7 - i)));
  unsigned char* begin = buf + 10 - len;
  begin[0] ^= kHeader[len][0];
  begin[1] ^= kHeader[len][1];
  dest.append(reinterpret_cast<const char*>(begin), len);
}

std::string encode_tensor_name_slice(const std::string& name, const SliceSpec& slice) {
  std::string key;
  oc_write_num_increasing(key, 0);
  oc_write_string(key, name);
  oc_write_num_increasing(key, (uint64_t)slice.size());
  for (const auto& d : slice) {
    oc_write_signed_num_increasing(key, d.second == -1 ? 0 : d.first);
    oc_write_signed_num_increasing(key, d.second);
  }
  return key;
}

bool decode_bundle_entry(const std::string& s, BundleEntry& e) {
  std::vector<PbField> fs;
  if (!pb_parse(s, fs)) return false;
  e = BundleEntry();
  for (const auto& f : fs) {
    if (f.field == 1) e.dtype = (int)f.v;
    else if (f.field == 4) e.offset = (int64_t)f.v;
    else if (f.field == 5) e.size = (int64_t)f.v;
    else if (f.field == 6) e.crc = crc_unmask((uint32_t)f.v);
    else if (f.field == 7) {
      std::vector<PbField> exts;
      if (!pb_parse(f.s, exts)) return false;
      SliceSpec sl;
      for (const auto& x : exts) {
        if (x.field != 1) continue;
        std::vector<PbField> ee;
        if (!pb_parse(x.s, ee)) return false;
        int64_t start = 0, length = -1;
        for (const auto& y : ee) {
          if (y.field == 1) start = (int64_t)y.v;
          else if (y.field == 2) length = (int64_t)y.v;
        }
        sl.emplace_back(start, length);
      }
      e.slices.push_back(sl);
    }
    else if (f.field == 2) {
      std::vector<PbField> dims;
      if (!pb_parse(f.s, dims)) return false;
      for (const auto& d : dims) {
        if (d.field != 2) continue;
        std::vector<PbField> dd;
        if (!pb_parse(d.s, dd)) return false;
        int64_t size = 0;
        for (const auto& x : dd) if (x.field == 1) size = (int64_t)x.v;
        e.shape.push_back(size);
      }
    }
  }
  return true;
}

void BundleWriter::add(const std::string& name, int dtype, const std::vector<int64_t>& shape,
                       const std::string& bytes) {
  if (name.empty()) throw std::runtime_error("bundle: empty tensor name is reserved for the header");
  BundleEntry e;
  e.dtype = dtype;
  e.shape = shape;
  e.size = (int64_t)bytes.size();
  e.crc = crc32c(bytes.data(), bytes.size());
  items_[name] = {e, bytes};
}

void BundleWriter::add_slice(const std::string& name, int dtype, const std::vector<int64_t>& full_shape,
                             const SliceSpec& slice, const std::string& bytes) {
  if (name.empty()) throw std::runtime_error("bundle: empty tensor name is reserved for the header");
  if (slice.size() != full_shape.size()) throw std::runtime_error("bundle: slice rank != tensor rank");
  auto it = items_.find(name);
  if (it == items_.end()) {
    BundleEntry full;
    full.dtype = dtype;
    full.shape = full_shape;
    it = items_.emplace(name, std::make_pair(full, std::string())).first;
  } else if (it->second.first.dtype != dtype || it->second.first.shape != full_shape || !it->second.second.empty()) {
    throw std::runtime_error("bundle: slice of " + name + " disagrees with its other slices");
  }
  it->second.first.slices.push_back(slice);
  std::vector<int64_t> shape;
  for (size_t d = 0; d < slice.size(); ++d) {
    if (slice[d].second != -1 && (slice[d].first < 0 || slice[d].first + slice[d].second > full_shape[d]))
      throw std::runtime_error("bundle: slice of " + name + " out of range");
    shape.push_back(slice[d].second == -1 ? full_shape[d] : slice[d].second);
  }
  add(encode_tensor_name_slice(name, slice), dtype, shape, bytes);
}

static void write_file_atomic(const std::string& path, const std::string& contents) {
  const std::string tmp = path + ".tempstate";
  {
    std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
    if (!f) throw std::runtime_error("cannot open " + tmp);
    f.write(contents.data(), (std::streamsize)contents.size());
    if (!f) throw std::runtime_error("write failed: " + tmp);
  }
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("rename failed: " + path);
}

void BundleWriter::finish(const std::string& prefix) {
  std::string data;
  std::vector<std::pair<std::string, std::string>> kv;
  // header: num_shards=1, endianness=LITTLE (0, omitted), version{producer=1}
  PbWriter ver;
  ver.u64(1, 1);
  PbWriter hdr;
  hdr.u64(1, 1);
  hdr.bytes(3, ver.buf);
  kv.emplace_back("", hdr.buf);
  for (auto& it : items_) {  // std::map: sorted bytewise
    BundleEntry e = it.second.first;
    if (!it.second.second.empty() || e.slices.empty()) {
      e.offset = (int64_t)data.size();
      data += it.second.second;
    }
    kv.emplace_back(it.first, encode_bundle_entry(e));
  }
  write_file_atomic(prefix + ".data-00000-of-00001", data);
  write_file_atomic(prefix + ".index", sstable_build(kv));
}

static bool read_file(const std::string& path, std::string& out, std::string* err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) { if (err) *err = "cannot open " + path; return false; }
  std::ostringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return true;
}

bool bundle_read_index(const std::string& prefix, std::map<std::string, BundleEntry>& out, std::string* err) {
  std::string file;
  if (!read_file(prefix + ".index", file, err)) return false;
  std::vector<std::pair<std::string, std::string>> kv;
  if (!sstable_parse(file, kv, err)) return false;
  for (const auto& e : kv) {
    if (e.first.empty()) continue;  // header
    BundleEntry be;
    if (!decode_bundle_entry(e.second, be)) { if (err) *err = "bad entry for " + e.first; return false; }
    out[e.first] = be;
  }
  return true;
}

bool bundle_read_tensor(const std::string& prefix, const BundleEntry& e, std::string& bytes, std::string* err) {
  std::ifstream f(prefix + ".data-00000-of-00001", std::ios::binary);
  if (!f) { if (err) *err = "cannot open data file"; return false; }
  f.seekg(e.offset);
  bytes.resize((size_t)e.size);
  f.read(&bytes[0], e.size);
  if (!f) { if (err) *err = "short read"; return false; }
  if (crc32c(bytes.data(), bytes.size()) != e.crc) { if (err) *err = "tensor crc mismatch"; return false; }
  return true;
}

// ================================================================= events
std::string tfrecord_frame(const std::string& data) {
  std::string out;
  std::string len;
  put_fixed64(len, (uint64_t)data.size());
  out += len;
  put_fixed32(out, crc_mask(crc32c(len.data(), 8)));
  out += data;
  put_fixed32(out, crc_mask(crc32c(data.data(), data.size())));
  return out;
}

bool tfrecord_read_all(const std::string& path, std::vector<std::string>& recs, std::string* err) {
  std::string f;
  if (!read_file(path, f, err)) return false;
  size_t p = 0;
  while (p + 12 <= f.size()) {
    const uint64_t n = get_fixed64(f.data() + p);
    if (crc_mask(crc32c(f.data() + p, 8)) != get_fixed32(f.data() + p + 8)) { if (err) *err = "length crc"; return false; }
    if (p + 12 + n + 4 > f.size()) { if (err) *err = "truncated record"; return false; }
    const char* d = f.data() + p + 12;
    if (crc_mask(crc32c(d, n)) != get_fixed32(d + n)) { if (err) *err = "data crc"; return false; }
    recs.emplace_back(d, n);
    p += 12 + n + 4;
  }
  return true;
}

std::string event_file_version(double wall_time) {
  PbWriter w;
  w.f64(1, wall_time);
  w.bytes(3, "brain.Event:2");
  return w.buf;
}

std::string event_scalars(double wall_time, int64_t step, const std::vector<std::pair<std::string, float>>& tags) {
  PbWriter summary;
  for (const auto& t : tags) {
    PbWriter v;
    v.bytes(1, t.first);
    v.f32(2, t.second);
    summary.bytes(1, v.buf);
  }
  PbWriter w;
  w.f64(1, wall_time);
  w.i64(2, step);
  w.bytes(5, summary.buf);
  return w.buf;
}

std::string event_graph(double wall_time, const std::string& graph_def) {
  PbWriter w;
  w.f64(1, wall_time);
  w.bytes(4, graph_def);
  return w.buf;
}

std::string event_meta_graph(double wall_time, const std::string& mg) {
  PbWriter w;
  w.f64(1, wall_time);
  w.bytes(9, mg);
  return w.buf;
}

static std::string attr_entry(const std::string& key, const std::string& attr_value) {
  PbWriter e;
  e.bytes(1, key);
  e.bytes(2, attr_value);
  return e.buf;
}

std::string graph_def_for_variables(const std::vector<std::tuple<std::string, int, std::vector<int64_t>>>& vars) {
  PbWriter g;
  for (const auto& v : vars) {
    PbWriter node;
    node.bytes(1, std::get<0>(v));
    node.bytes(2, "VariableV2");
    PbWriter dt;
    dt.u64(6, (uint64_t)std::get<1>(v));
    PbWriter shp;
    shp.bytes(7, encode_shape(std::get<2>(v)));
    PbWriter empty_s;
    empty_s.bytes(2, "");
    node.bytes(5, attr_entry("container", empty_s.buf));
    node.bytes(5, attr_entry("dtype", dt.buf));
    node.bytes(5, attr_entry("shape", shp.buf));
    node.bytes(5, attr_entry("shared_name", empty_s.buf));
    g.bytes(1, node.buf);
  }
  PbWriter versions;
  versions.u64(1, 26);  // TF 1.11 GraphDef producer version
  g.bytes(4, versions.buf);
  return g.buf;
}

std::string meta_graph_def(const std::string& graph_def, const std::string& tf_version) {
  PbWriter info;
  info.bytes(5, tf_version);
  PbWriter saver;
  saver.bytes(1, "save/Const:0");
  saver.bytes(2, "save/control_dependency:0");
  saver.bytes(3, "save/restore_all");
  saver.u64(4, 5);
  saver.f32(6, 10000.0f);
  saver.u64(7, 2);  // SaverDef.V2
  PbWriter m;
  m.bytes(1, info.buf);
  m.bytes(2, graph_def);
  m.bytes(3, saver.buf);
  return m.buf;
}

// ================================================================= MNIST
bool idx_read(const std::string& path, IdxArray& out, std::string* err) {
  gzFile f = gzopen(path.c_str(), "rb");  // transparently reads uncompressed files too
  if (!f) { if (err) *err = "cannot open " + path; return false; }
  std::string buf;
  char chunk[1 << 16];
  int n;
  while ((n = gzread(f, chunk, sizeof(chunk))) > 0) buf.append(chunk, n);
  gzclose(f);
  if (buf.size() < 4) { if (err) *err = "short idx file"; return false; }
  const uint8_t* b = (const uint8_t*)buf.data();
  if (b[0] != 0 || b[1] != 0 || b[2] != 0x08) { if (err) *err = "unsupported idx type (need uint8)"; return false; }
  const int nd = b[3];
  if (buf.size() < 4 + 4 * (size_t)nd) { if (err) *err = "short idx header"; return false; }
  out.dims.clear();
  size_t total = 1;
  for (int i = 0; i < nd; ++i) {
    const uint32_t d = (uint32_t)b[4 + 4 * i] << 24 | (uint32_t)b[5 + 4 * i] << 16 | (uint32_t)b[6 + 4 * i] << 8 |
                       (uint32_t)b[7 + 4 * i];
    out.dims.push_back(d);
    total *= d;
  }
  const size_t hdr = 4 + 4 * (size_t)nd;
  if (buf.size() < hdr + total) { if (err) *err = "truncated idx payload"; return false; }
  out.data.assign(b + hdr, b + hdr + total);
  return true;
}

void EpochBatcher::shuffle() {
  perm_.resize(n_);
  for (int64_t i = 0; i < n_; ++i) perm_[i] = (int32_t)i;
  std::shuffle(perm_.begin(), perm_.end(), rng_);
}

std::vector<int32_t> EpochBatcher::next(int64_t batch) {
  if (!started_) {
    shuffle();
    started_ = true;
  }
  std::vector<int32_t> out;
  out.reserve(batch);
  if (pos_ + batch > n_) {
    // rest of this epoch, then reshuffle and take the remainder of the batch
    ++epochs_;
    for (int64_t i = pos_; i < n_; ++i) out.push_back(perm_[i]);
    const int64_t rest = batch - (n_ - pos_);
    shuffle();
    for (int64_t i = 0; i < rest; ++i) out.push_back(perm_[i]);
    pos_ = rest;
  } else {
    for (int64_t i = pos_; i < pos_ + batch; ++i) out.push_back(perm_[i]);
    pos_ += batch;
  }
  return out;
}

}  // namespace dtfe_rt

// Native runtime pieces that replace TF 1.11's C++ runtime for the reference
// scripts' side effects:
//   * crc32c (SSE4.2) + TF's masked crc
//   * protobuf wire-format encoders/decoders for the handful of TF messages
//     we emit (BundleHeaderProto, BundleEntryProto, TensorShapeProto, Event,
//     Summary, VersionDef, a minimal MetaGraphDef)
//   * LevelDB-format SSTable writer/reader (TF's tensor-bundle .index)
//   * tensor-bundle V2 writer/reader (model.ckpt-N.{index,data-00000-of-00001})
//   * TFRecord framing (events.out.tfevents.*)
//   * MNIST idx(.gz) reader and the epoch-shuffling batcher of
//     tensorflow/examples/tutorials/mnist (next_batch semantics)
#pragma once
#include <cstdint>
#include <map>
#include <random>
#include <string>
#include <vector>

namespace dtfe_rt {

// ---------------------------------------------------------------- crc32c
uint32_t crc32c_extend(uint32_t init, const void* data, size_t n);
inline uint32_t crc32c(const void* data, size_t n) { return crc32c_extend(0, data, n); }
inline uint32_t crc_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
inline uint32_t crc_unmask(uint32_t m) {
  uint32_t rot = m - 0xa282ead8u;
  return ((rot >> 17) | (rot << 15));
}

// ---------------------------------------------------------------- protobuf
struct PbWriter {
  std::string buf;
  void varint(uint64_t v);
  void key(int field, int wt) { varint((uint64_t)(field << 3 | wt)); }
  void u64(int field, uint64_t v) { key(field, 0); varint(v); }
  void i64(int field, int64_t v) { u64(field, (uint64_t)v); }
  void bytes(int field, const std::string& s) { key(field, 2); varint(s.size()); buf += s; }
  void fixed32(int field, uint32_t v);
  void fixed64(int field, uint64_t v);
  void f32(int field, float v);
  void f64(int field, double v);
};

struct PbField {
  int field, wt;
  uint64_t v;       // varint / fixed value
  std::string s;    // length-delimited payload
};
// Parses one message level; returns false on malformed input.
bool pb_parse(const std::string& msg, std::vector<PbField>& out);

// ---------------------------------------------------------------- encoding
void put_fixed32(std::string& s, uint32_t v);
void put_fixed64(std::string& s, uint64_t v);
void put_varint(std::string& s, uint64_t v);
bool get_varint(const char*& p, const char* end, uint64_t& v);
uint32_t get_fixed32(const char* p);
uint64_t get_fixed64(const char* p);

// ---------------------------------------------------------------- SSTable
// LevelDB table format (TF core/lib/io/table_builder): uncompressed blocks,
// restart interval 16, masked-crc block trailers, 48-byte footer.
std::string sstable_build(const std::vector<std::pair<std::string, std::string>>& sorted_kv,
                          size_t block_size = 262144);
bool sstable_parse(const std::string& file, std::vector<std::pair<std::string, std::string>>& out,
                   std::string* err);

// ---------------------------------------------------------------- bundle
// TF DataType enum values for the dtypes we save
enum TfDtype : int { DT_FLOAT = 1, DT_DOUBLE = 2, DT_INT32 = 3, DT_UINT8 = 4, DT_INT64 = 9, DT_BFLOAT16 = 14 };

// one TensorSliceProto: per dimension (start, length); length -1 = the full extent
typedef std::vector<std::pair<int64_t, int64_t>> SliceSpec;

struct BundleEntry {
  int dtype = 0;
  std::vector<int64_t> shape;
  int64_t offset = 0, size = 0;
  uint32_t crc = 0;  // unmasked crc32c of the bytes
  // a partitioned variable's full-tensor entry (BundleEntryProto.slices): metadata only, the data of
  // each slice lives under the key encode_tensor_name_slice(name, slice)
  std::vector<SliceSpec> slices;
};

// TF's checkpoint::EncodeTensorNameSlice (tensorflow/core/util/saved_tensor_slice_util.cc): the
// OrderedCode key of one slice of a partitioned tensor - 0, the name, the rank, then (start, length)
// per dimension as signed increasing numbers (a full extent: start 0, length -1)
std::string encode_tensor_name_slice(const std::string& name, const SliceSpec& slice);

class BundleWriter {
 public:
  void add(const std::string& name, int dtype, const std::vector<int64_t>& shape, const std::string& bytes);
  // one slice of a partitioned tensor (BundleWriter::AddSlice): records the slice in the full
  // tensor's entry and stores the slice's data under its encoded key
  void add_slice(const std::string& name, int dtype, const std::vector<int64_t>& full_shape, const SliceSpec& slice,
                 const std::string& bytes);
  // writes <prefix>.index and <prefix>.data-00000-of-00001 (atomically via .tempstate files)
  void finish(const std::string& prefix);

 private:
  std::map<std::string, std::pair<BundleEntry, std::string>> items_;
};

bool bundle_read_index(const std::string& prefix, std::map<std::string, BundleEntry>& out, std::string* err);
bool bundle_read_tensor(const std::string& prefix, const BundleEntry& e, std::string& bytes, std::string* err);

std::string encode_bundle_entry(const BundleEntry& e);
bool decode_bundle_entry(const std::string& s, BundleEntry& e);

// ---------------------------------------------------------------- events
std::string tfrecord_frame(const std::string& data);
// parse all records of a TFRecord file; returns false if a crc mismatches
bool tfrecord_read_all(const std::string& path, std::vector<std::string>& recs, std::string* err);
std::string event_file_version(double wall_time);
std::string event_scalars(double wall_time, int64_t step, const std::vector<std::pair<std::string, float>>& tags);
std::string event_graph(double wall_time, const std::string& graph_def);
std::string event_meta_graph(double wall_time, const std::string& meta_graph_def);

// Minimal GraphDef / MetaGraphDef describing the saved variables (VariableV2
// nodes with dtype/shape attrs) + a SaverDef pointing at the checkpoint ops.
std::string graph_def_for_variables(const std::vector<std::tuple<std::string, int, std::vector<int64_t>>>& vars);
std::string meta_graph_def(const std::string& graph_def, const std::string& tf_version);

// ---------------------------------------------------------------- MNIST
struct IdxArray {
  std::vector<int64_t> dims;
  std::vector<uint8_t> data;  // uint8 idx payload (type 0x08)
};
bool idx_read(const std::string& path, IdxArray& out, std::string* err);  // .gz or raw

// tensorflow.contrib.learn DataSet.next_batch(batch, shuffle=True) index semantics:
// shuffle at the first call, stitch the tail of an epoch with the head of the
// next (freshly shuffled) one.
class EpochBatcher {
 public:
  EpochBatcher(int64_t n, uint64_t seed) : n_(n), rng_(seed) {}
  std::vector<int32_t> next(int64_t batch);
  int64_t epochs_completed() const { return epochs_; }

 private:
  void shuffle();
  int64_t n_;
  std::mt19937_64 rng_;
  std::vector<int32_t> perm_;
  int64_t pos_ = 0, epochs_ = 0;
  bool started_ = false;
};

}  // namespace dtfe_rt

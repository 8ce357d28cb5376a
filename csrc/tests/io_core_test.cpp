// Standalone ASan + UBSan driver for the torch-free ImageNet reader core (csrc/io/io_core.h),
// built and run by scripts/sanitize_host.sh.  Exercises well-formed and hostile inputs: every
// truncation of a tf.Example, truncated and bit-flipped JPEGs, crop and pad geometry, and the
// decode thread pool.  Exit status 0 = all checks passed and no sanitizer report.
#include <cstdio>
#include <cstdlib>
#include <random>

#include "io/io_core.h"

using namespace pddl_io;

static int fails = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) { std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } \
  } while (0)

static std::vector<uint8_t> encode_jpeg(int H, int W, int C) {
  jpeg_compress_struct ci;
  jpeg_error_mgr je;
  ci.err = jpeg_std_error(&je);
  jpeg_create_compress(&ci);
  unsigned char* mem = nullptr;
  unsigned long n = 0;
  jpeg_mem_dest(&ci, &mem, &n);
  ci.image_width = W; ci.image_height = H; ci.input_components = C;
  ci.in_color_space = C == 3 ? JCS_RGB : JCS_GRAYSCALE;
  jpeg_set_defaults(&ci);
  jpeg_set_quality(&ci, 95, TRUE);
  jpeg_start_compress(&ci, TRUE);
  std::vector<uint8_t> row((size_t)W * C);
  while (ci.next_scanline < ci.image_height) {
    const int y = (int)ci.next_scanline;
    for (int x = 0; x < W; ++x)
      for (int c = 0; c < C; ++c) row[(size_t)x * C + c] = (uint8_t)((x * 3 + y * 2 + c * 40) & 255);
    JSAMPROW rp = row.data();
    jpeg_write_scanlines(&ci, &rp, 1);
  }
  jpeg_finish_compress(&ci);
  std::vector<uint8_t> out(mem, mem + n);
  free(mem);
  jpeg_destroy_compress(&ci);
  return out;
}

static void varint(std::vector<uint8_t>& o, uint64_t v) {
  do { uint8_t b = v & 0x7F; v >>= 7; o.push_back(v ? (b | 0x80) : b); } while (v);
}
static std::vector<uint8_t> field(int num, const std::vector<uint8_t>& payload) {
  std::vector<uint8_t> o;
  varint(o, (uint64_t)(num << 3) | 2);
  varint(o, payload.size());
  o.insert(o.end(), payload.begin(), payload.end());
  return o;
}
static std::vector<uint8_t> bytes_of(const std::string& s) { return std::vector<uint8_t>(s.begin(), s.end()); }
static std::vector<uint8_t> cat(std::vector<uint8_t> a, const std::vector<uint8_t>& b) {
  a.insert(a.end(), b.begin(), b.end());
  return a;
}
static std::vector<uint8_t> example(const std::vector<uint8_t>& jpg, int64_t label) {
  auto entry = [](const std::string& k, const std::vector<uint8_t>& feat) {
    return field(1, cat(field(1, bytes_of(k)), field(2, feat)));
  };
  std::vector<uint8_t> lab;
  varint(lab, (uint64_t)label);
  return field(1, cat(entry("image", field(1, field(1, jpg))), entry("label", field(3, field(1, lab)))));
}

int main() {
  // CRC32C check value (RFC 3720): crc32c("123456789") = 0xE3069283
  const char* nine = "123456789";
  CHECK(crc32c(reinterpret_cast<const uint8_t*>(nine), 9) == 0xE3069283u);

  const std::vector<uint8_t> rgb = encode_jpeg(45, 70, 3), gray = encode_jpeg(20, 30, 1);
  // crop (45x70 -> 32x32: offsets (6, 19)) and pad (20x30 -> 32x32: offsets (6, 1))
  std::vector<uint8_t> out(32 * 32 * 3, 77);
  decode_crop_pad(rgb.data(), rgb.size(), 32, out.data());
  const int ref = (19 * 3 + 6 * 2) & 255;   // top-left of the crop, channel 0 (JPEG-lossy)
  CHECK(std::abs((int)out[0] - ref) < 12);
  decode_crop_pad(gray.data(), gray.size(), 32, out.data());
  CHECK(out[0] == 0 && out[(5 * 32 + 31) * 3] == 0);            // padded rows / columns are zero
  CHECK(out[(6 * 32 + 1) * 3] == out[(6 * 32 + 1) * 3 + 1]);    // grayscale expanded to RGB

  // tf.Example round trip + every truncation (must never read out of bounds)
  const std::vector<uint8_t> ex = example(rgb, 917);
  const uint8_t* img = nullptr;
  size_t img_n = 0;
  int64_t label = -1;
  CHECK(parse_example(ex.data(), ex.size(), &img, &img_n, &label, "image", "label"));
  CHECK(label == 917 && img_n == rgb.size() && std::memcmp(img, rgb.data(), img_n) == 0);
  int ok_prefixes = 0;
  for (size_t n = 0; n < ex.size(); ++n) {
    std::vector<uint8_t> t(ex.begin(), ex.begin() + n);   // exact-size heap copy: ASan sees overreads
    ok_prefixes += parse_example(t.data(), t.size(), &img, &img_n, &label, "image", "label");
  }
  CHECK(ok_prefixes == 0);

  // hostile JPEG bytes: truncations and bit flips decode or throw, never fault
  std::mt19937 rng(7);
  int threw = 0, decoded = 0;
  for (int trial = 0; trial < 200; ++trial) {
    std::vector<uint8_t> j = rgb;
    if (trial % 2) j.resize(rng() % j.size());
    else for (int k = 0; k < 4; ++k) j[rng() % j.size()] ^= (uint8_t)(1u << (rng() % 8));
    try {
      decode_crop_pad(j.data(), j.size(), 24, out.data());
      ++decoded;
    } catch (const std::runtime_error&) {
      ++threw;
    }
  }
  CHECK(threw + decoded == 200 && threw > 0);

  // thread pool: all tasks run once, first error propagates
  Pool pool(4);
  std::vector<std::atomic<int>> hits(1000);
  pool.run(1000, [&](int64_t i) { hits[i].fetch_add(1); });
  int all_once = 1;
  for (auto& h : hits) all_once &= h.load() == 1;
  CHECK(all_once);
  bool caught = false;
  try {
    pool.run(50, [&](int64_t i) { if (i == 17) throw std::runtime_error("boom"); });
  } catch (const std::runtime_error& e) {
    caught = std::string(e.what()) == "boom";
  }
  CHECK(caught);

  // concurrent callers (serialized by the pool) writing plain, non-atomic per-call buffers that
  // the caller reads after run() returns: the worker -> caller hand-off must order those
  // writes (ThreadSanitizer checks it in scripts/sanitize_host.sh); decodes run on the pool as
  // in the reader
  std::vector<std::thread> callers;
  std::atomic<int> bad{0};
  for (int c = 0; c < 4; ++c)
    callers.emplace_back([&, c] {
      for (int rep = 0; rep < 20; ++rep) {
        std::vector<int> vals(64, 0);
        std::vector<uint8_t> imgs(8 * 24 * 24 * 3);
        pool.run(64, [&](int64_t i) {
          vals[i] = (int)i * (c + 1);
          if (i < 8) decode_crop_pad(rgb.data(), rgb.size(), 24, imgs.data() + i * 24 * 24 * 3);
        });
        for (int i = 0; i < 64; ++i) bad += vals[i] != i * (c + 1);
        for (int i = 1; i < 8; ++i) bad += std::memcmp(imgs.data(), imgs.data() + i * 24 * 24 * 3, 24 * 24 * 3) != 0;
      }
    });
  for (auto& t : callers) t.join();
  CHECK(bad.load() == 0);

  std::printf("io_core_test: %s (%d hostile JPEGs threw, %d decoded)\n", fails ? "FAILED" : "ok", threw, decoded);
  return fails ? 1 : 0;
}

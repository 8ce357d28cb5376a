// Torch-free core of the native ImageNet reader (csrc/io/imagenet_io.cpp): masked CRC32C of
// the TFRecord framing, a minimal protobuf walker for tf.Example, libjpeg decode fused with
// tf.image.resize_with_crop_or_pad, and the decode thread pool.  Kept free of torch so the
// sanitizer driver (csrc/tests/io_core_test.cpp) builds it with ASan + UBSan standalone.
#pragma once
#include <fcntl.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <csetjmp>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

extern "C" {
#include <jpeglib.h>
}

namespace pddl_io {

// ---------------------------------------------------------------------------- CRC32C
inline uint32_t crc_table[256];
struct CrcInit {
  CrcInit() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0x82F63B78u ^ (c >> 1) : c >> 1;
      crc_table[i] = c;
    }
  }
};
inline CrcInit crc_init;
inline uint32_t crc32c(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}
inline uint32_t masked_crc(const uint8_t* p, size_t n) {
  const uint32_t c = crc32c(p, n);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

// ------------------------------------------------------------------- protobuf (tf.Example)
struct PB {
  const uint8_t* p;
  const uint8_t* e;
  bool varint(uint64_t* v) {
    uint64_t r = 0;
    for (int s = 0; s < 64 && p < e; s += 7) {
      const uint8_t b = *p++;
      r |= (uint64_t)(b & 0x7F) << s;
      if (!(b & 0x80)) { *v = r; return true; }
    }
    return false;
  }
  // next field: tag, wire type; for length-delimited fields sub = [start, end)
  bool next(uint32_t* field, int* wt, PB* sub, uint64_t* val) {
    if (p >= e) return false;
    uint64_t key;
    if (!varint(&key)) return false;
    *field = (uint32_t)(key >> 3);
    *wt = (int)(key & 7);
    switch (*wt) {
      case 0: return varint(val);
      case 1: if (e - p < 8) return false; p += 8; return true;
      case 5: if (e - p < 4) return false; p += 4; return true;
      case 2: {
        uint64_t len;
        if (!varint(&len) || (uint64_t)(e - p) < len) return false;
        sub->p = p; sub->e = p + len; p += len;
        return true;
      }
      default: return false;
    }
  }
};

// Extract the "image" bytes and the "label" int64 from a serialized tf.Example.
inline bool parse_example(const uint8_t* data, size_t n, const uint8_t** img, size_t* img_n, int64_t* label,
                   const std::string& image_key, const std::string& label_key) {
  PB ex{data, data + n};
  uint32_t f; int wt; PB sub{}; uint64_t v;
  bool got_img = false, got_lab = false;
  while (ex.next(&f, &wt, &sub, &v)) {
    if (f != 1 || wt != 2) continue;                 // Example.features
    PB feats = sub;
    PB entry{};
    while (feats.next(&f, &wt, &entry, &v)) {
      if (f != 1 || wt != 2) continue;               // Features.feature (map entry)
      std::string key;
      PB feature{};
      bool has_val = false;
      PB e2 = entry, s2{};
      while (e2.next(&f, &wt, &s2, &v)) {
        if (f == 1 && wt == 2) key.assign((const char*)s2.p, s2.e - s2.p);
        else if (f == 2 && wt == 2) { feature = s2; has_val = true; }
      }
      if (!has_val) continue;
      PB kind{};
      while (feature.next(&f, &wt, &kind, &v)) {
        if (wt != 2) continue;
        if (f == 1 && key == image_key) {             // BytesList { repeated bytes value = 1 }
          PB bl = kind, b{};
          while (bl.next(&f, &wt, &b, &v))
            if (f == 1 && wt == 2) { *img = b.p; *img_n = b.e - b.p; got_img = true; break; }
        } else if (f == 3 && key == label_key) {      // Int64List { repeated int64 value = 1 }
          PB il = kind, b{};
          while (il.next(&f, &wt, &b, &v)) {
            if (f == 1 && wt == 0) { *label = (int64_t)v; got_lab = true; break; }
            if (f == 1 && wt == 2) {                  // packed
              PB pk = b;
              uint64_t x;
              if (pk.varint(&x)) { *label = (int64_t)x; got_lab = true; }
              break;
            }
          }
        }
      }
    }
  }
  return got_img && got_lab;
}

// ------------------------------------------------------------------------------ JPEG
struct JErr {
  jpeg_error_mgr pub;
  jmp_buf jb;
  char msg[JMSG_LENGTH_MAX];
};
inline void jerr_silent(j_common_ptr) {}   // corrupt-data warnings: recoverable, not printed
inline void jerr_exit(j_common_ptr c) {
  JErr* e = reinterpret_cast<JErr*>(c->err);
  (*c->err->format_message)(c, e->msg);
  longjmp(e->jb, 1);
}

// Decode and write tf.image.resize_with_crop_or_pad(img, S, S) into out[S][S][3].
inline void decode_crop_pad(const uint8_t* buf, size_t n, int S, uint8_t* out) {
  jpeg_decompress_struct ci;
  JErr je;
  ci.err = jpeg_std_error(&je.pub);
  je.pub.error_exit = jerr_exit;
  je.pub.output_message = jerr_silent;
  std::vector<uint8_t> row;
  if (setjmp(je.jb)) {
    jpeg_destroy_decompress(&ci);
    throw std::runtime_error(std::string("jpeg decode: ") + je.msg);
  }
  jpeg_create_decompress(&ci);
  jpeg_mem_src(&ci, const_cast<unsigned char*>(buf), (unsigned long)n);
  jpeg_read_header(&ci, TRUE);
  const bool cmyk = ci.jpeg_color_space == JCS_CMYK || ci.jpeg_color_space == JCS_YCCK;
  if (cmyk) ci.out_color_space = JCS_CMYK;
  else if (ci.num_components == 1) ci.out_color_space = JCS_GRAYSCALE;
  else ci.out_color_space = JCS_RGB;
  jpeg_start_decompress(&ci);
  const int H = (int)ci.output_height, W = (int)ci.output_width, C = ci.output_components;
  // crop offsets (larger dims) and pad offsets (smaller dims), as resize_with_crop_or_pad
  const int cy = H > S ? (H - S) / 2 : 0, cx = W > S ? (W - S) / 2 : 0;
  const int py = S > H ? (S - H) / 2 : 0, px = S > W ? (S - W) / 2 : 0;
  const int ch = H < S ? H : S, cw = W < S ? W : S;
  std::memset(out, 0, (size_t)S * S * 3);
  row.resize((size_t)W * C);
  const bool adobe_inverted = cmyk && ci.saw_Adobe_marker;
  // rows past the crop window are never needed: stop there and abort the decompressor (the
  // center crop of a 375-row ImageNet image leaves ~20% of the rows undecoded)
  const int y_end = cy + ch;
  while ((int)ci.output_scanline < y_end) {
    const int y = (int)ci.output_scanline;
    JSAMPROW rp = row.data();
    jpeg_read_scanlines(&ci, &rp, 1);
    if (y < cy || y >= cy + ch) continue;
    uint8_t* o = out + ((size_t)(y - cy + py) * S + px) * 3;
    const uint8_t* r = row.data() + (size_t)cx * C;
    if (C == 3) {
      std::memcpy(o, r, (size_t)cw * 3);
    } else if (C == 1) {
      for (int x = 0; x < cw; ++x) o[3 * x] = o[3 * x + 1] = o[3 * x + 2] = r[x];
    } else {   // CMYK -> RGB
      for (int x = 0; x < cw; ++x) {
        int c = r[4 * x], m = r[4 * x + 1], yy = r[4 * x + 2], k = r[4 * x + 3];
        if (!adobe_inverted) { c = 255 - c; m = 255 - m; yy = 255 - yy; k = 255 - k; }
        o[3 * x] = (uint8_t)(c * k / 255);
        o[3 * x + 1] = (uint8_t)(m * k / 255);
        o[3 * x + 2] = (uint8_t)(yy * k / 255);
      }
    }
  }
  if ((int)ci.output_scanline < H) jpeg_abort_decompress(&ci);
  else jpeg_finish_decompress(&ci);
  jpeg_destroy_decompress(&ci);
}

// ------------------------------------------------------------------------- thread pool
class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 0; i < (n > 0 ? n : 1); ++i) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // run fn(i) for i in [0, n) on the pool; rethrows the first error.  Calls from several
  // threads are serialized (one job in flight).
  void run(int64_t n, const std::function<void(int64_t)>& fn) {
    std::lock_guard<std::mutex> job(run_mu_);
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn; n_ = n; next_.store(0); done_ = 0; err_.clear(); ++gen_;
    }
    cv_.notify_all();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return done_ == (int)th_.size(); });
    fn_ = nullptr;
    if (!err_.empty()) throw std::runtime_error(err_);
  }

 private:
  void loop() {
    uint64_t seen = 0;
    while (true) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      while (true) {
        const int64_t i = next_.fetch_add(1);
        if (i >= n_) break;
        try {
          (*fn_)(i);
        } catch (const std::exception& e) {
          std::lock_guard<std::mutex> lk(mu_);
          if (err_.empty()) err_ = e.what();
        }
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        ++done_;
      }
      done_cv_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  bool stop_ = false;
  uint64_t gen_ = 0;
  int done_ = 0;
  const std::function<void(int64_t)>* fn_ = nullptr;
  int64_t n_ = 0;
  std::atomic<int64_t> next_{0};
  std::string err_;
};

inline bool pread_all(int fd, uint8_t* dst, size_t n, off_t off) {
  while (n > 0) {
    const ssize_t r = pread(fd, dst, n, off);
    if (r <= 0) return false;
    dst += r; n -= (size_t)r; off += r;
  }
  return true;
}

}  // namespace pddl_io

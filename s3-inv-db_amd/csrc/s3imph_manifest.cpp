// s3imph_manifest.cpp — manifest.json of an index directory (optional
// part): the SHA-256 and size of every index file, as format.WriteManifest /
// ReadManifest / VerifyManifest do (/root/reference/pkg/format/manifest.go:14-155), called
// by IndexBuilder.Finalize once every file is written (pkg/extsort/indexbuild.go:429-432).
//
// Host code: SHA-256 over a file is one sequential chain, so it stays on the CPU.  The
// files are hashed in parallel (one thread per file, where the reference walks them one
// by one), each with 4 MiB pread chunks and the x86 SHA extensions when the CPU has them
// (a portable FIPS 180-4 loop otherwise).  The JSON text is the one Go's
// json.MarshalIndent(manifest, "", "  ") writes: fields in struct order, the files map
// with sorted keys, created_at in RFC 3339 with nanoseconds (trailing zeros trimmed).
#include <fcntl.h>
#include <immintrin.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "s3imph.h"
#include "s3imph_internal.h"

namespace s3imph {
namespace {

constexpr uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// FIPS 180-4 compression, one 64-byte block at a time.
void blocks_portable(uint32_t st[8], const uint8_t* p, size_t nb) {
  for (; nb; --nb, p += 64) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
      w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
      const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; ++i) {
      const uint32_t t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + kK[i] + w[i];
      const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      h = g;
      g = f;
      f = e;
      e = d + t1;
      d = c;
      c = b;
      b = a;
      a = t1 + t2;
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
    st[4] += e;
    st[5] += f;
    st[6] += g;
    st[7] += h;
  }
}

// The same compression on the SHA extensions: the state lives as (ABEF, CDGH), each
// sha256rnds2 does two rounds, and the message schedule rotates through four registers.
__attribute__((target("sha,sse4.1,ssse3"))) void blocks_shani(uint32_t st[8], const uint8_t* p, size_t nb) {
  const __m128i kMask = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
  __m128i tmp = _mm_loadu_si128(reinterpret_cast<const __m128i*>(&st[0]));
  __m128i s1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(&st[4]));
  tmp = _mm_shuffle_epi32(tmp, 0xB1);                // CDAB
  s1 = _mm_shuffle_epi32(s1, 0x1B);                  // EFGH
  __m128i s0 = _mm_alignr_epi8(tmp, s1, 8);          // ABEF
  s1 = _mm_blend_epi16(s1, tmp, 0xF0);               // CDGH
  for (; nb; --nb, p += 64) {
    const __m128i abef = s0, cdgh = s1;
    __m128i w[4];
#pragma GCC unroll 16
    for (int g = 0; g < 16; ++g) {
      if (g < 4) w[g] = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 16 * g)), kMask);
      __m128i msg = _mm_add_epi32(w[g & 3], _mm_loadu_si128(reinterpret_cast<const __m128i*>(&kK[4 * g])));
      s1 = _mm_sha256rnds2_epu32(s1, s0, msg);
      if (g >= 3 && g <= 14) {
        const __m128i t = _mm_alignr_epi8(w[g & 3], w[(g + 3) & 3], 4);
        w[(g + 1) & 3] = _mm_sha256msg2_epu32(_mm_add_epi32(w[(g + 1) & 3], t), w[g & 3]);
      }
      msg = _mm_shuffle_epi32(msg, 0x0E);
      s0 = _mm_sha256rnds2_epu32(s0, s1, msg);
      if (g >= 1 && g <= 12) w[(g + 3) & 3] = _mm_sha256msg1_epu32(w[(g + 3) & 3], w[g & 3]);
    }
    s0 = _mm_add_epi32(s0, abef);
    s1 = _mm_add_epi32(s1, cdgh);
  }
  tmp = _mm_shuffle_epi32(s0, 0x1B);                 // FEBA
  s1 = _mm_shuffle_epi32(s1, 0xB1);                  // DCHG
  s0 = _mm_blend_epi16(tmp, s1, 0xF0);               // DCBA
  s1 = _mm_alignr_epi8(s1, tmp, 8);                  // HGFE
  _mm_storeu_si128(reinterpret_cast<__m128i*>(&st[0]), s0);
  _mm_storeu_si128(reinterpret_cast<__m128i*>(&st[4]), s1);
}

struct Sha256 {
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t buf[64];
  size_t nbuf = 0;
  uint64_t total = 0;
  bool ni = false;
  explicit Sha256(bool use_ni) : ni(use_ni) {}
  void blocks(const uint8_t* p, size_t nb) { ni ? blocks_shani(st, p, nb) : blocks_portable(st, p, nb); }
  void update(const uint8_t* p, size_t n) {
    total += n;
    if (nbuf) {
      const size_t t = std::min(n, 64 - nbuf);
      std::memcpy(buf + nbuf, p, t);
      nbuf += t;
      p += t;
      n -= t;
      if (nbuf == 64) {
        blocks(buf, 1);
        nbuf = 0;
      }
    }
    if (n >= 64) {
      blocks(p, n / 64);
      p += n & ~size_t(63);
      n &= 63;
    }
    if (n) {
      std::memcpy(buf, p, n);
      nbuf = n;
    }
  }
  std::string hex() {
    const uint64_t bits = total * 8;
    uint8_t pad[72] = {0x80};
    const size_t padlen = (nbuf < 56 ? 56 - nbuf : 120 - nbuf);
    for (int i = 0; i < 8; ++i) pad[padlen + i] = (uint8_t)(bits >> (56 - 8 * i));
    update(pad, padlen + 8);
    static const char* d = "0123456789abcdef";
    std::string s(64, '0');
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 4; ++j) {
        const uint8_t b = (uint8_t)(st[i] >> (24 - 8 * j));
        s[8 * i + 2 * j] = d[b >> 4];
        s[8 * i + 2 * j + 1] = d[b & 15];
      }
    return s;
  }
};

bool have_shani() {
  static const bool v = __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1");
  return v;
}

// checksumFile (manifest.go:140-155): SHA-256 hex of the whole file.
int checksum_file(const std::string& path, bool use_ni, std::string* hex, std::string* msg) {
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) {
    *msg = "open file: " + std::string(std::strerror(errno));
    return S3IMPH_ERR_IO;
  }
  Sha256 h(use_ni);
  std::vector<uint8_t> chunk(4u << 20);
  for (uint64_t off = 0;;) {
    const ssize_t r = ::pread(fd, chunk.data(), chunk.size(), (off_t)off);
    if (r < 0) {
      if (errno == EINTR) continue;
      *msg = "read file: " + std::string(std::strerror(errno));
      ::close(fd);
      return S3IMPH_ERR_IO;
    }
    if (r == 0) break;
    h.update(chunk.data(), (size_t)r);
    off += (uint64_t)r;
  }
  ::close(fd);
  *hex = h.hex();
  return S3IMPH_OK;
}

// The index files WriteManifest looks for (manifest.go:44-57); absent ones are skipped.
const char* const kIndexFiles[] = {"subtree_end.u64",   "depth.u32",           "object_count.u64",
                                   "total_bytes.u64",   "max_depth_in_subtree.u32", "depth_offsets.u64",
                                   "depth_positions.u64", "mph.bin",           "mph_fp.u64",
                                   "mph_pos.u64",       "prefix_blob.bin",     "prefix_offsets.u64"};

struct FileInfo {
  int64_t size = 0;
  std::string checksum;
};

// Hash the named files of dir on one thread each.
int checksum_files(const std::string& dir, const std::vector<std::string>& names, std::vector<std::string>* sums,
                   std::string* msg) {
  const bool ni = have_shani();
  sums->assign(names.size(), "");
  std::vector<int> rcs(names.size(), S3IMPH_OK);
  std::vector<std::string> errs(names.size());
  std::vector<std::thread> th;
  for (size_t i = 0; i < names.size(); ++i)
    th.emplace_back([&, i] { rcs[i] = checksum_file(dir + "/" + names[i], ni, &(*sums)[i], &errs[i]); });
  for (auto& t : th) t.join();
  for (size_t i = 0; i < names.size(); ++i)
    if (rcs[i] != S3IMPH_OK) {
      *msg = "checksum " + names[i] + ": " + errs[i];
      return rcs[i];
    }
  return S3IMPH_OK;
}

// time.Now().UTC() as encoding/json writes it (RFC 3339, nanoseconds without trailing zeros).
std::string rfc3339_now() {
  timespec ts{};
  clock_gettime(CLOCK_REALTIME, &ts);
  tm t{};
  gmtime_r(&ts.tv_sec, &t);
  char b[64];
  std::strftime(b, sizeof b, "%Y-%m-%dT%H:%M:%S", &t);
  std::string s = b;
  if (ts.tv_nsec) {
    char f[16];
    std::snprintf(f, sizeof f, ".%09ld", ts.tv_nsec);
    std::string fs = f;
    while (fs.back() == '0') fs.pop_back();
    s += fs;
  }
  return s + "Z";
}

// ---- a small reader for the manifest's JSON (objects, strings, integers) ------------
struct Json {
  const std::string& s;
  size_t i = 0;
  bool ok = true;
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\r' || s[i] == '\t')) ++i;
  }
  bool eat(char c) {
    ws();
    if (i < s.size() && s[i] == c) {
      ++i;
      return true;
    }
    return false;
  }
  std::string str() {
    ws();
    std::string out;
    if (i >= s.size() || s[i] != '"') {
      ok = false;
      return out;
    }
    for (++i; i < s.size() && s[i] != '"'; ++i) {
      if (s[i] == '\\' && i + 1 < s.size()) ++i;
      out += s[i];
    }
    if (i >= s.size()) ok = false;
    ++i;
    return out;
  }
  // skips any value; returns it as text when it is a string or a number
  std::string value() {
    ws();
    if (i >= s.size()) {
      ok = false;
      return "";
    }
    if (s[i] == '"') return str();
    if (s[i] == '{' || s[i] == '[') {
      const char open = s[i], close = open == '{' ? '}' : ']';
      int depth = 0;
      bool in_str = false;
      for (; i < s.size(); ++i) {
        if (in_str) {
          if (s[i] == '\\') ++i;
          else if (s[i] == '"') in_str = false;
        } else if (s[i] == '"') {
          in_str = true;
        } else if (s[i] == open) {
          ++depth;
        } else if (s[i] == close && --depth == 0) {
          ++i;
          return "";
        }
      }
      ok = false;
      return "";
    }
    const size_t b = i;
    while (i < s.size() && s[i] != ',' && s[i] != '}' && s[i] != ']' && s[i] != ' ' && s[i] != '\n') ++i;
    return s.substr(b, i - b);
  }
};

int read_manifest_files(const std::string& dir, std::map<std::string, FileInfo>* files, std::string* msg) {
  const std::string path = dir + "/manifest.json";
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) {
    *msg = "read manifest: open " + path + ": " + std::strerror(errno);
    return S3IMPH_ERR_IO;
  }
  std::string text;
  char b[1 << 16];
  for (size_t r; (r = std::fread(b, 1, sizeof b, f)) > 0;) text.append(b, r);
  std::fclose(f);
  Json j{text};
  bool saw_files = false;
  if (!j.eat('{')) j.ok = false;
  while (j.ok && !j.eat('}')) {
    const std::string key = j.str();
    if (!j.eat(':')) j.ok = false;
    if (!j.ok) break;
    if (key == "files") {
      saw_files = true;
      if (!j.eat('{')) {
        j.ok = false;
        break;
      }
      while (j.ok && !j.eat('}')) {
        const std::string name = j.str();
        if (!j.eat(':') || !j.eat('{')) {
          j.ok = false;
          break;
        }
        FileInfo fi;
        while (j.ok && !j.eat('}')) {
          const std::string k2 = j.str();
          if (!j.eat(':')) j.ok = false;
          const std::string v = j.value();
          if (k2 == "size") fi.size = std::strtoll(v.c_str(), nullptr, 10);
          else if (k2 == "checksum") fi.checksum = v;
          j.eat(',');
        }
        (*files)[name] = fi;
        j.eat(',');
      }
    } else {
      j.value();
    }
    j.eat(',');
  }
  if (!j.ok || !saw_files) {
    *msg = "unmarshal manifest: malformed " + path;
    return S3IMPH_ERR_FORMAT;
  }
  return S3IMPH_OK;
}

}  // namespace

int write_manifest(const std::string& dir, uint64_t node_count, uint32_t max_depth, std::string* msg) {
  std::vector<std::string> names;
  std::vector<int64_t> sizes;
  for (const char* nm : kIndexFiles) {
    struct stat sb{};
    const std::string path = dir + "/" + nm;
    if (::stat(path.c_str(), &sb) != 0) {
      if (errno == ENOENT) continue;  // optional file
      *msg = std::string("stat ") + nm + ": " + std::strerror(errno);
      return S3IMPH_ERR_IO;
    }
    names.push_back(nm);
    sizes.push_back((int64_t)sb.st_size);
  }
  std::vector<std::string> sums;
  int rc = checksum_files(dir, names, &sums, msg);
  if (rc != S3IMPH_OK) return rc;
  std::map<std::string, FileInfo> files;  // encoding/json writes map keys sorted
  for (size_t i = 0; i < names.size(); ++i) files[names[i]] = FileInfo{sizes[i], sums[i]};
  std::string out = "{\n  \"version\": 1,\n  \"created_at\": \"" + rfc3339_now() + "\",\n  \"node_count\": " +
                    std::to_string(node_count) + ",\n  \"max_depth\": " + std::to_string(max_depth) +
                    ",\n  \"files\": {";
  if (files.empty()) {
    out += "}";
  } else {
    bool first = true;
    for (const auto& kv : files) {
      out += first ? "\n" : ",\n";
      first = false;
      out += "    \"" + kv.first + "\": {\n      \"size\": " + std::to_string(kv.second.size) +
             ",\n      \"checksum\": \"" + kv.second.checksum + "\"\n    }";
    }
    out += "\n  }";
  }
  out += "\n}";
  // writeFileSync (manifest.go:157-177): create, write, fsync, close
  const std::string path = dir + "/manifest.json";
  const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) {
    *msg = "write manifest: create file: " + std::string(std::strerror(errno));
    return S3IMPH_ERR_IO;
  }
  size_t done = 0;
  while (done < out.size()) {
    const ssize_t w = ::write(fd, out.data() + done, out.size() - done);
    if (w < 0) {
      if (errno == EINTR) continue;
      *msg = "write manifest: write file: " + std::string(std::strerror(errno));
      ::close(fd);
      return S3IMPH_ERR_IO;
    }
    done += (size_t)w;
  }
  if (::fsync(fd) != 0 || ::close(fd) != 0) {
    *msg = "write manifest: sync file: " + std::string(std::strerror(errno));
    return S3IMPH_ERR_IO;
  }
  return S3IMPH_OK;
}

int verify_manifest(const std::string& dir, std::string* msg) {
  std::map<std::string, FileInfo> files;
  int rc = read_manifest_files(dir, &files, msg);
  if (rc != S3IMPH_OK) return rc;
  std::vector<std::string> names;
  for (const auto& kv : files) {
    struct stat sb{};
    if (::stat((dir + "/" + kv.first).c_str(), &sb) != 0) {
      *msg = "file " + kv.first + ": " + std::strerror(errno);
      return S3IMPH_ERR_IO;
    }
    if ((int64_t)sb.st_size != kv.second.size) {
      *msg = "file " + kv.first + ": size mismatch (got " + std::to_string((int64_t)sb.st_size) + ", want " +
             std::to_string(kv.second.size) + ")";
      return S3IMPH_ERR_FORMAT;
    }
    names.push_back(kv.first);
  }
  std::vector<std::string> sums;
  rc = checksum_files(dir, names, &sums, msg);
  if (rc != S3IMPH_OK) return rc;
  for (size_t i = 0; i < names.size(); ++i)
    if (sums[i] != files[names[i]].checksum) {
      *msg = "file " + names[i] + ": checksum mismatch";
      return S3IMPH_ERR_FORMAT;
    }
  return S3IMPH_OK;
}

}  // namespace s3imph

extern "C" {

int s3imph_write_manifest(const char* out_dir, uint64_t node_count, uint32_t max_depth, char* err, size_t errlen) {
  if (!out_dir) return S3IMPH_ERR_INVALID;
  std::string msg;
  const int rc = s3imph::write_manifest(out_dir, node_count, max_depth, &msg);
  if (rc != S3IMPH_OK) s3imph::set_err(err, errlen, "write manifest: " + msg);
  return rc;
}

int s3imph_verify_manifest(const char* dir, char* err, size_t errlen) {
  if (!dir) return S3IMPH_ERR_INVALID;
  std::string msg;
  const int rc = s3imph::verify_manifest(dir, &msg);
  if (rc != S3IMPH_OK) s3imph::set_err(err, errlen, msg);
  return rc;
}

int s3imph_sha256_file(const char* path, int portable, char hex_out[65], char* err, size_t errlen) {
  if (!path || !hex_out) return S3IMPH_ERR_INVALID;
  std::string hex, msg;
  const int rc = s3imph::checksum_file(path, !portable && s3imph::have_shani(), &hex, &msg);
  if (rc != S3IMPH_OK) {
    s3imph::set_err(err, errlen, msg);
    return rc;
  }
  std::memcpy(hex_out, hex.c_str(), 65);
  return S3IMPH_OK;
}

}  // extern "C"

// librodio.so — host-side data and checkpoint I/O behind include/rodio.h (no device code).
//
// What the reference gets from TensorFlow's C++ runtime on its input side:
//   * CRC32C (Castagnoli), masked as TF masks it, for TFRecord framing
//     (tensorflow/core/lib/io/record_reader.cc) and tensor-bundle entries
//     (tensorflow/core/util/tensor_bundle) — ref dataset/pascalvoc_common.py:71-72 reads with
//     tf.TFRecordReader, train.py:155-158/282 restores bundles with tf.train.Saver;
//   * the TFRecord scan: every record's payload offset and length, both checksums verified.
// Slice-by-8 table CRC (portable; ~1-2 GB/s per thread), no intrinsics.
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

namespace {

thread_local std::string g_err;

void set_err(const char* fmt, const char* a, long b) {
  char buf[512];
  snprintf(buf, sizeof buf, fmt, a, b);
  g_err = buf;
}

struct Tables {
  uint32_t t[8][256];
  Tables() {
    const uint32_t poly = 0x82F63B78u;  // reflected Castagnoli polynomial
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
  }
};
const Tables kT;

uint32_t crc_extend(uint32_t crc, const uint8_t* p, size_t n) {
  uint32_t c = ~crc;
  while (n && ((uintptr_t)p & 7)) {
    c = kT.t[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
    --n;
  }
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    uint32_t lo = (uint32_t)v ^ c, hi = (uint32_t)(v >> 32);
    c = kT.t[7][lo & 0xFF] ^ kT.t[6][(lo >> 8) & 0xFF] ^ kT.t[5][(lo >> 16) & 0xFF] ^ kT.t[4][lo >> 24] ^
        kT.t[3][hi & 0xFF] ^ kT.t[2][(hi >> 8) & 0xFF] ^ kT.t[1][(hi >> 16) & 0xFF] ^ kT.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = kT.t[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
  return ~c;
}

inline uint32_t masked(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }

inline uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

}  // namespace

extern "C" {

const char* rodio_last_error(void) { return g_err.c_str(); }

int rodio_abi_version(void) { return 1; }

unsigned rodio_crc32c_extend(unsigned crc, const void* data, size_t n) {
  return crc_extend(crc, (const uint8_t*)data, n);
}

unsigned rodio_masked_crc32c(const void* data, size_t n) {
  return masked(crc_extend(0, (const uint8_t*)data, n));
}

// Scan a TFRecord file: record i's payload starts at offsets[i] and is lengths[i] bytes.
// Returns the number of records (fills the first min(count, cap) entries), or -1 with
// rodio_last_error() set on a truncated file or a checksum mismatch.  verify_data=0 checks
// only the length checksums (the payload CRC costs one pass over the file).
long rodio_tfrecord_scan(const char* path, long* offsets, long* lengths, long cap, int verify_data) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    set_err("rodio_tfrecord_scan: cannot open %s (errno %ld)", path, errno);
    return -1;
  }
  // the file size bounds every record length: a crafted header with a valid length CRC but a
  // huge length must not reach the allocation or the seek (std::bad_alloc through extern "C"
  // would abort the host process; (long)len could overflow)
  if (fseek(f, 0, SEEK_END) != 0) {
    set_err("rodio_tfrecord_scan: cannot seek in %s (errno %ld)", path, errno);
    fclose(f);
    return -1;
  }
  const long fsize = ftell(f);
  if (fsize < 0 || fseek(f, 0, SEEK_SET) != 0) {
    set_err("rodio_tfrecord_scan: cannot size %s (errno %ld)", path, errno);
    fclose(f);
    return -1;
  }
  long count = 0, pos = 0;
  uint8_t hdr[12];
  std::string buf;
  for (;;) {
    size_t got = fread(hdr, 1, 12, f);
    if (got == 0) break;
    if (got != 12) {
      set_err("rodio_tfrecord_scan: %s truncated in a record header at byte %ld", path, pos);
      fclose(f);
      return -1;
    }
    uint64_t len;
    memcpy(&len, hdr, 8);
    if (masked(crc_extend(0, hdr, 8)) != rd32(hdr + 8)) {
      set_err("rodio_tfrecord_scan: %s corrupted record length at byte %ld", path, pos);
      fclose(f);
      return -1;
    }
    long data_off = pos + 12;
    if (len > (uint64_t)(fsize - data_off) || (uint64_t)(fsize - data_off) - len < 4) {
      set_err("rodio_tfrecord_scan: %s truncated: the record at byte %ld claims a length past the end of the file", path, pos);
      fclose(f);
      return -1;
    }
    uint8_t foot[4];
    if (verify_data) {
      buf.resize(len);
      if (fread(&buf[0], 1, len, f) != len || fread(foot, 1, 4, f) != 4) {
        set_err("rodio_tfrecord_scan: %s truncated in the record at byte %ld", path, pos);
        fclose(f);
        return -1;
      }
      if (masked(crc_extend(0, (const uint8_t*)buf.data(), len)) != rd32(foot)) {
        set_err("rodio_tfrecord_scan: %s corrupted record data at byte %ld", path, pos);
        fclose(f);
        return -1;
      }
    } else if (fseek(f, (long)len, SEEK_CUR) != 0 || fread(foot, 1, 4, f) != 4) {
      set_err("rodio_tfrecord_scan: %s truncated in the record at byte %ld", path, pos);
      fclose(f);
      return -1;
    }
    if (count < cap) {
      offsets[count] = data_off;
      lengths[count] = (long)len;
    }
    ++count;
    pos = data_off + (long)len + 4;
  }
  fclose(f);
  return count;
}

}  // extern "C"

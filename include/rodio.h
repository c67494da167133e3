/* librodio.so — host-side data and checkpoint I/O of the CLIs (no device code).
 *
 * Replaces what the reference takes from TensorFlow's runtime on its input side:
 *   - tf.TFRecordReader framing + CRC32C checks (ref dataset/pascalvoc_common.py:71-72,
 *     read through slim's DatasetDataProvider at utils/data_pileline_tools.py:18-69);
 *   - the CRC32C of tf.train.Saver tensor bundles (ref train.py:155-158, 176, 282;
 *     evaluate.py:221-224), used by rod/checkpoint.py to verify imported variables.
 * Bound by rod/io_native.py (ctypes).  Return conventions: counts >= 0 or -1 with the
 * message in rodio_last_error() (thread-local).
 */
#ifndef RODIO_H
#define RODIO_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

int rodio_abi_version(void);
const char* rodio_last_error(void);

/* CRC32C (Castagnoli) of n bytes continuing from crc (0 to start); unmasked. */
unsigned rodio_crc32c_extend(unsigned crc, const void* data, size_t n);

/* TF's masked CRC32C: ((c >> 15) | (c << 17)) + 0xa282ead8 of the CRC32C c of the bytes. */
unsigned rodio_masked_crc32c(const void* data, size_t n);

/* Record i's payload: bytes [offsets[i], offsets[i] + lengths[i]) of the file.  Returns the
 * record count (first min(count, cap) entries filled) or -1 (truncated / bad checksum).
 * verify_data: also check every payload's CRC (one pass over the file). */
long rodio_tfrecord_scan(const char* path, long* offsets, long* lengths, long cap, int verify_data);

#ifdef __cplusplus
}
#endif
#endif /* RODIO_H */

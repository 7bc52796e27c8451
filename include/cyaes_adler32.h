/*
 * cyaes_adler32.h -- Adler-32 on the MI355X.
 * Library: libcyaes.so.
 *
 * Same function as cyclone::adler32 (source/cyCrypt/crypt/cyr_adler32.h:33,
 * cyr_adler32.cpp:66-133): the zlib Adler-32 update, modulo 65521, with the
 * reference's own edge rule -- a NULL buffer or len == 0 returns
 * INITIAL_ADLER (1) whatever the running value (cyr_adler32.cpp:72-73; zlib
 * would return the running value for len == 0).  Callers in the reference:
 * RingBuf::checksum (cyc_ring_buf.cpp:365-387) and the filetransfer sample's
 * fragment CRC (ft_client.cpp:219, ft_server.cpp:181).
 *
 * HBM-bound byte work: the kernels read each byte once and form the two
 * sums from per-dword v_dot4_u32_u8 partials (sum of bytes, position-weighted
 * sum), reduced modulo 65521 -- no sequential dependence between bytes.
 */
#ifndef CYAES_ADLER32_H
#define CYAES_ADLER32_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CYAES_INITIAL_ADLER 1u /* INITIAL_ADLER, cyr_adler32.h:12 */

/* Batch of independent buffers (device memory; any byte offsets/lengths):
 *   d_out[k] = adler32(d_adler_in ? d_adler_in[k] : INITIAL_ADLER,
 *                      d_buf + d_offsets[k], d_nbytes[k]).
 * Asynchronous on `stream`. */
int cyaes_gpu_adler32_batch(const uint8_t* d_buf, const uint64_t* d_offsets, const uint64_t* d_nbytes,
                            const uint32_t* d_adler_in, uint32_t* d_out, uint64_t n, void* stream);

/* One (large) device buffer, reduced by the whole GPU:
 *   *out = adler32(adler, d_buf, nbytes).  Synchronous (waits on `stream`). */
int cyaes_gpu_adler32(const uint8_t* d_buf, uint64_t nbytes, uint32_t adler, uint32_t* out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* CYAES_ADLER32_H */

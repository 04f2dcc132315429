// sigma.hpp — sparse public matrix H and the per-edge sigma generator.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pvac_hip.h"

namespace pvhip {

// H stored column-sparse: rows[c * width + k] (u16) for k < counts[c].
struct sigma_tables {
    uint16_t* rows = nullptr;
    uint32_t* counts = nullptr;
    // m_bits == 8192, x_col_wt == 128 and full columns only: the same rows re-encoded for k_sigma's
    // fast column expansion, (r & 31) | (r >> 5) << 7 (bits 5..14 are the image byte offset)
    uint16_t* rows_fast = nullptr;
    // the same default-geometry columns as 208 byte increments of R = (r >> 5) | (r & 31) << 8
    // (see k_sigma.hip flip_cols_delta); null when unavailable
    uint8_t* rows_delta = nullptr;
    uint32_t width = 0;
    uint32_t n_cols = 0;
    bool full = false;   // every column has exactly `width` rows (no padding: k_sigma drops its guards)
    bool ready = false;
};

void sigma_tables_free(sigma_tables& T);
// device copy of src for a context on dst_dev (peer copies when the devices differ); synchronous
hipError_t sigma_tables_clone(sigma_tables& dst, const sigma_tables& src, int dst_dev, int src_dev, hipStream_t st);
// host SHA-256 over a contiguous buffer
void sha256_host(const uint8_t* p, size_t n, uint8_t out[32]);
// from a HOST dense H (n_bits columns x ceil(m_bits/64) words); synchronous
hipError_t sigma_tables_from_dense(sigma_tables& T, const pvac_hip_params& prm, const uint64_t* H_host, hipStream_t st);
// gen_H (crypto/matrix.hpp:191-251) on the device; digest computed on the host; synchronous
hipError_t sigma_tables_generate(sigma_tables& T, const pvac_hip_params& prm, uint8_t digest[32], hipStream_t st);
// sigma for every edge slot of X (salt of edge slot e = salts[e], or salts[e_off + salt_pos[e]])
hipError_t launch_sigma(const sigma_tables& T, const pvac_hip_params& prm, const pvac_ct_batch& X,
                        const uint64_t* salts, const uint32_t* salt_pos, int num_cus, hipStream_t st);

}  // namespace pvhip

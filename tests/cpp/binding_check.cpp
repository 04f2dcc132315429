// binding_check.cpp — compile/link check of the INTEGRATION.md §2 reference-side binding against the
// REAL reference headers (/root/reference/include, pvac-hfhe 0.1.0): each function below is the body
// a maintainer puts under PVAC_USE_MI355X in ops/arithmetic.hpp, ops/encrypt.hpp and
// ops/decrypt.hpp, instantiated on pvac::PubKey / SecKey / Cipher / Fp (core/types.hpp:72-139,
// core/field.hpp, core/bitvec.hpp:9-11). Built and linked by tests/test_binding.py only where the
// reference exists (this container); never run, never shipped.
#include <pvac/pvac.hpp>
#include <pvac_hip.hpp>

#include <type_traits>

namespace binding {

using pvac::Cipher;
using pvac::Fp;
using pvac::PubKey;
using pvac::SecKey;

Cipher ct_add(const PubKey& pk, const Cipher& A, const Cipher& B) { return pvac_hip::ct_add(pk, A, B); }    // arithmetic.hpp:12
Cipher ct_sub(const PubKey& pk, const Cipher& A, const Cipher& B) { return pvac_hip::ct_sub(pk, A, B); }    // :43
Cipher ct_scale(const PubKey& pk, const Cipher& A, const Fp& s) { return pvac_hip::ct_scale(pk, A, s); }    // :33
Cipher ct_mul(const PubKey& pk, const Cipher& A, const Cipher& B) { return pvac_hip::ct_mul(pk, A, B); }    // :47
Cipher ct_neg(const PubKey& pk, const Cipher& A) { return pvac_hip::ct_neg(pk, A); }                         // :39
Cipher ct_div_const(const PubKey& pk, const Cipher& A, const Fp& k) { return pvac_hip::ct_div_const(pk, A, k); } // :108
Cipher enc_value(const PubKey& pk, const SecKey& sk, uint64_t v) {                                          // encrypt.hpp:289
    return pvac_hip::enc_value<Cipher>(pk, sk, v);
}
Cipher enc_value_depth(const PubKey& pk, const SecKey& sk, uint64_t v, int d) {                           // encrypt.hpp:281
    return pvac_hip::enc_value_depth<Cipher>(pk, sk, v, d);
}
Cipher enc_zero_depth(const PubKey& pk, const SecKey& sk, int d) { return pvac_hip::enc_zero_depth<Cipher>(pk, sk, d); } // :293
Fp dec_value(const PubKey& pk, const SecKey& sk, const Cipher& C) { return pvac_hip::dec_value(pk, sk, C); } // decrypt.hpp:62
std::vector<Cipher> load_cts(const std::vector<uint8_t>& b) { return pvac_hip::load_cts_bytes<Cipher>(b); }
std::vector<uint8_t> save_cts(const std::vector<Cipher>& c) { return pvac_hip::save_cts_bytes(c); }

static_assert(std::is_same<decltype(pvac_hip::dec_value(std::declval<const PubKey&>(), std::declval<const SecKey&>(),
                                                        std::declval<const Cipher&>())),
                           Fp>::value,
              "dec_value returns the reference's Fp");

}  // namespace binding

int main(int argc, char**) {
    // link check only: reference every binding so nothing is discarded
    volatile void* keep[] = {(void*)&binding::ct_add,    (void*)&binding::ct_sub,    (void*)&binding::ct_scale,
                             (void*)&binding::ct_mul,    (void*)&binding::enc_value, (void*)&binding::dec_value,
                             (void*)&binding::load_cts,  (void*)&binding::save_cts,
                             (void*)&binding::enc_value_depth, (void*)&binding::enc_zero_depth};
    return argc > 99 ? (int)(uintptr_t)keep[0] : 0;
}

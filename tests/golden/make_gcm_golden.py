"""Generate tests/golden/gcm.json: AES-GCM known answers from the host's OpenSSL libcrypto.

replicat's cipher adapter calls `cryptography`'s AESGCM (replicat/utils/adapters.py:127-134),
a binding of OpenSSL's EVP AES-GCM.  `cryptography` is not installed in this image, but OpenSSL's
libcrypto is, so the expected outputs come from the same EVP calls made through ctypes
(EncryptInit with the GCM cipher, SET_IVLEN, EncryptUpdate, EncryptFinal, GET_TAG): exactly what
AESGCM(key).encrypt(nonce, data, None) returns.  Run in the build container:

    python tests/golden/make_gcm_golden.py

Inputs are seeded (random.Random(seed).randbytes), so the file stays small: a case stores its
plaintext as hex (short ones) or as (pt_seed, pt_len), and its output C || T as hex (up to 4 KiB)
or as SHA-256 plus the tag.
"""
import ctypes
import ctypes.util
import hashlib
import json
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, 'gcm.json')

_c = ctypes.CDLL(ctypes.util.find_library('crypto') or 'libcrypto.so.3')
_vp = ctypes.c_void_p
for _name in ('EVP_aes_128_gcm', 'EVP_aes_192_gcm', 'EVP_aes_256_gcm', 'EVP_CIPHER_CTX_new'):
    getattr(_c, _name).restype = _vp
    getattr(_c, _name).argtypes = []
_c.EVP_CIPHER_CTX_free.argtypes = [_vp]
_c.EVP_EncryptInit_ex.argtypes = [_vp, _vp, _vp, ctypes.c_char_p, ctypes.c_char_p]
_c.EVP_CIPHER_CTX_ctrl.argtypes = [_vp, ctypes.c_int, ctypes.c_int, _vp]
_c.EVP_EncryptUpdate.argtypes = [_vp, _vp, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
_c.EVP_EncryptFinal_ex.argtypes = [_vp, _vp, ctypes.POINTER(ctypes.c_int)]
EVP_CTRL_GCM_SET_IVLEN, EVP_CTRL_GCM_GET_TAG = 0x9, 0x10


def openssl_gcm_encrypt(key, iv, pt):
    """AESGCM(key).encrypt(iv, pt, None) = C || T through OpenSSL's EVP interface."""
    cipher = {16: _c.EVP_aes_128_gcm, 24: _c.EVP_aes_192_gcm, 32: _c.EVP_aes_256_gcm}[len(key)]()
    ctx = _c.EVP_CIPHER_CTX_new()
    try:
        assert _c.EVP_EncryptInit_ex(ctx, cipher, None, None, None) == 1
        assert _c.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_SET_IVLEN, len(iv), None) == 1
        assert _c.EVP_EncryptInit_ex(ctx, None, None, key, iv) == 1
        out = ctypes.create_string_buffer(len(pt) + 16)
        n = ctypes.c_int(0)
        if pt:
            assert _c.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), pt, len(pt)) == 1
        fin, m = ctypes.create_string_buffer(32), ctypes.c_int(0)
        assert _c.EVP_EncryptFinal_ex(ctx, fin, ctypes.byref(m)) == 1
        assert n.value + m.value == len(pt)
        tag = ctypes.create_string_buffer(16)
        assert _c.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_GET_TAG, 16, tag) == 1
        return out.raw[:n.value] + fin.raw[:m.value] + tag.raw
    finally:
        _c.EVP_CIPHER_CTX_free(ctx)


def plaintext(case):
    if 'pt' in case:
        return bytes.fromhex(case['pt'])
    return random.Random(case['pt_seed']).randbytes(case['pt_len'])


def cases():
    rnd = random.Random(0x6763)
    out = []
    # SP 800-38D / McGrew-Viega test cases 1, 2, 13, 14 (all-zero key and IV)
    for kb in (16, 32):
        for n in (0, 16):
            out.append({'name': f'zero_k{kb}_p{n}', 'key': bytes(kb).hex(), 'iv': bytes(12).hex(),
                        'pt': bytes(n).hex()})
    # the reference's own adapter test input (replicat/tests/test_adapters.py:21-26)
    out.append({'name': 'adapter_test', 'key': b'<key>'.ljust(32, b'\x00').hex(),
                'iv': bytes(range(12)).hex(), 'pt': b'<some data>'.hex()})
    lens = [1, 15, 16, 17, 31, 32, 33, 100, 255, 256, 257, 1000, 4095, 4096, 4097, 16383, 16384,
            16385, 16400, 32773, 65536, 100003]
    seed = 1000
    for kb in (16, 24, 32):
        for n in [0] + lens:
            ivs = (12, 8, 16, 13, 60, 128) if n in (0, 17, 16385) else (12,)
            for ivn in ivs:
                seed += 1
                case = {'name': f'k{kb}_iv{ivn}_p{n}', 'key': rnd.randbytes(kb).hex(),
                        'iv': rnd.randbytes(ivn).hex()}
                if n <= 64:
                    case['pt'] = random.Random(seed).randbytes(n).hex()
                else:
                    case['pt_seed'], case['pt_len'] = seed, n
                out.append(case)
    # chunk-sized: a 1 MiB + 3 chunk and replicat's largest chunk (max_length 5,120,000)
    for kb, n in ((32, (1 << 20) + 3), (32, 5_120_000), (16, 5_120_000)):
        seed += 1
        out.append({'name': f'big_k{kb}_p{n}', 'key': rnd.randbytes(kb).hex(),
                    'iv': rnd.randbytes(12).hex(), 'pt_seed': seed, 'pt_len': n})
    return out


def main():
    res = []
    for case in cases():
        ct = openssl_gcm_encrypt(bytes.fromhex(case['key']), bytes.fromhex(case['iv']), plaintext(case))
        if len(ct) <= 4096 + 16:
            case['out'] = ct.hex()
        else:
            case['out_sha256'] = hashlib.sha256(ct).hexdigest()
            case['tag'] = ct[-16:].hex()
        res.append(case)
    with open(OUT, 'w') as f:
        json.dump({'source': 'OpenSSL libcrypto EVP AES-GCM via ctypes (what cryptography.AESGCM '
                             'binds); tests/golden/make_gcm_golden.py', 'cases': res}, f, indent=1)
    print(f'{len(res)} cases -> {OUT}')


if __name__ == '__main__':
    main()

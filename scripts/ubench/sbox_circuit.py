"""A bitsliced AES S-box circuit (XOR / AND gates over 8 bit planes), generated from the tower
field GF(((2^2)^2)^2) and checked against the S-box table on all 256 inputs; emits the C body
that scripts/ubench/aes_bitslice.hip includes (round 6, VERDICT r5 item 6: a bitsliced AES-CTR
measured against the T-table kernel).

    python scripts/ubench/sbox_circuit.py > scripts/ubench/aes_sbox_gen.h

Construction (Canright's tower, polynomial bases): GF(4) = GF(2)[W]/(W^2+W+1),
GF(16) = GF(4)[Z]/(Z^2+Z+N), GF(256) = GF(16)[Y]/(Y^2+Y+V), with N, V the first constants that
make the quadratics irreducible.  inv(a1 Y + a0) = (a1 d^-1) Y + (a0 + a1) d^-1 with
d = a1^2 V + a1 a0 + a0^2, the same one level down, and x^-1 = x^2 in GF(4).  The AES field maps
to the tower through x -> b for a root b of the AES polynomial; S(a) = (A M^-1) inv(M a) + 0x63.
The linear parts are reduced by Paar's greedy common-pair elimination; the compiler fuses the
rest into v_bitop3_b32 (three-input) instructions.  Not product code: a measurement."""
import itertools
import sys

AES_POLY = 0x11B


def gf256_mul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= AES_POLY
        b >>= 1
    return r


def sbox_table():
    inv = [0] * 256
    for a in range(1, 256):
        for b in range(1, 256):
            if gf256_mul(a, b) == 1:
                inv[a] = b
                break
    out = []
    for a in range(256):
        x = inv[a]
        s = 0x63
        for i in range(8):
            bit = ((x >> i) ^ (x >> ((i + 4) % 8)) ^ (x >> ((i + 5) % 8)) ^ (x >> ((i + 6) % 8)) ^
                   (x >> ((i + 7) % 8))) & 1
            s ^= bit << i
        out.append(s)
    return out


# ---- tower arithmetic on concrete integers (to find constants and the isomorphism)
def g4_mul(a, b):  # (a1 W + a0)(b1 W + b0), W^2 = W + 1
    a0, a1, b0, b1 = a & 1, a >> 1, b & 1, b >> 1
    hh = a1 & b1
    return ((hh ^ (a1 & b0) ^ (a0 & b1)) << 1) | (hh ^ (a0 & b0))


def g16_mul(a, b, N):  # (a1 Z + a0)(b1 Z + b0), Z^2 = Z + N
    a0, a1, b0, b1 = a & 3, a >> 2, b & 3, b >> 2
    hh = g4_mul(a1, b1)
    return ((hh ^ g4_mul(a1, b0) ^ g4_mul(a0, b1)) << 2) | (g4_mul(hh, N) ^ g4_mul(a0, b0))


def g256_mul(a, b, N, V):
    a0, a1, b0, b1 = a & 15, a >> 4, b & 15, b >> 4
    hh = g16_mul(a1, b1, N)
    return ((hh ^ g16_mul(a1, b0, N) ^ g16_mul(a0, b1, N)) << 4) | (g16_mul(hh, V, N) ^ g16_mul(a0, b0, N))


def constants():
    N = next(n for n in range(1, 4) if all(g4_mul(z, z) ^ z ^ n for z in range(4)))
    V = next(v for v in range(1, 16) if all(g16_mul(y, y, N) ^ y ^ v for y in range(16)))
    return N, V


def tower_pow(b, e, N, V):
    r = 1
    for _ in range(e):
        r = g256_mul(r, b, N, V)
    return r


def isomorphism(N, V):
    """M: AES polynomial basis -> tower (columns M[i] = b^i)."""
    for b in range(2, 256):
        # b must satisfy b^8 + b^4 + b^3 + b + 1 = 0
        p = [tower_pow(b, k, N, V) for k in range(9)]
        if p[8] ^ p[4] ^ p[3] ^ p[1] ^ p[0] == 0:
            cols = p[:8]
            # check multiplicativity on random pairs
            def m(x):
                r = 0
                for i in range(8):
                    if x >> i & 1:
                        r ^= cols[i]
                return r
            if all(m(gf256_mul(x, y)) == g256_mul(m(x), m(y), N, V) for x, y in
                   itertools.product(range(0, 256, 7), range(0, 256, 11))):
                return cols
    raise RuntimeError('no root')


def mat_apply(cols, x):
    r = 0
    for i in range(8):
        if x >> i & 1:
            r ^= cols[i]
    return r


def mat_inverse(cols):
    table = {mat_apply(cols, x): x for x in range(256)}
    return [table[1 << i] for i in range(8)]


# ---- symbolic circuit: a value is a frozenset of base-signal ids (their XOR)
class Circ:
    def __init__(self):
        self.ands = []  # (lin_a, lin_b) -> base signal 8 + k

    def AND(self, a, b):
        if not a or not b:
            return frozenset()
        self.ands.append((a, b))
        return frozenset([8 + len(self.ands) - 1])


def X(a, b):
    return a ^ b


def s4_mul(c, a, b):
    a0, a1 = a
    b0, b1 = b
    hh = c.AND(a1, b1)
    ll = c.AND(a0, b0)
    mm = c.AND(X(a0, a1), X(b0, b1))  # Karatsuba: a1b0 + a0b1 = mm + hh + ll
    return (X(hh, ll), X(mm, ll))


def s4_add(a, b):
    return (X(a[0], b[0]), X(a[1], b[1]))


def s4_sq(a):  # (a1 W + a0)^2 = a1 W + (a0 + a1)
    return (X(a[0], a[1]), a[1])


def s4_const_mul(a, n):  # multiply by the constant n in GF(4): linear
    a0, a1 = a
    # n * (a1 W + a0), via the basis images
    w = [(1, 0), (0, 1)]  # placeholders
    r0, r1 = frozenset(), frozenset()
    for bit, val in ((0, a0), (1, a1)):
        img = g4_mul(1 << bit, n)
        if img & 1:
            r0 = X(r0, val)
        if img & 2:
            r1 = X(r1, val)
    return (r0, r1)


def s16_mul(c, a, b, N):
    a0, a1 = a
    b0, b1 = b
    hh = s4_mul(c, a1, b1)
    ll = s4_mul(c, a0, b0)
    mm = s4_mul(c, s4_add(a0, a1), s4_add(b0, b1))
    hi = s4_add(mm, ll)  # a1b0 + a0b1 + hh = mm + ll
    lo = s4_add(s4_const_mul(hh, N), ll)
    return (lo, hi)


def s16_add(a, b):
    return (s4_add(a[0], b[0]), s4_add(a[1], b[1]))


def s16_const_mul(a, v, N):
    bits = [a[0][0], a[0][1], a[1][0], a[1][1]]
    out = [frozenset()] * 4
    for i in range(4):
        img = g16_mul(1 << i, v, N)
        for k in range(4):
            if img >> k & 1:
                out[k] = X(out[k], bits[i])
    return ((out[0], out[1]), (out[2], out[3]))


def s16_sq(a, N):
    bits = [a[0][0], a[0][1], a[1][0], a[1][1]]
    out = [frozenset()] * 4
    for i in range(4):
        img = g16_mul(1 << i, 1 << i, N)
        for k in range(4):
            if img >> k & 1:
                out[k] = X(out[k], bits[i])
    return ((out[0], out[1]), (out[2], out[3]))


def s16_inv(c, a, N):
    a0, a1 = a
    # d = a1^2 N + a1 a0 + a0^2 (GF(4)), inv = (a1 d^-1) Z + (a0 + a1) d^-1, d^-1 = d^2
    d = s4_add(s4_add(s4_const_mul(s4_sq(a1), N), s4_mul(c, a1, a0)), s4_sq(a0))
    di = s4_sq(d)
    return (s4_mul(c, s4_add(a0, a1), di), s4_mul(c, a1, di))


def s256_inv(c, a, N, V):
    a0, a1 = a
    d = s16_add(s16_add(s16_const_mul(s16_sq(a1, N), V, N), s16_mul(c, a1, a0, N)), s16_sq(a0, N))
    di = s16_inv(c, d, N)
    return (s16_mul(c, s16_add(a0, a1), di, N), s16_mul(c, a1, di, N))


def build():
    N, V = constants()
    M = isomorphism(N, V)
    Minv = mat_inverse(M)
    c = Circ()
    x = [frozenset([i]) for i in range(8)]  # input bits 0..7 (LSB first)
    t = [frozenset()] * 8  # t = M x
    for i in range(8):
        for k in range(8):
            if M[i] >> k & 1:
                t[k] = X(t[k], x[i])
    a = ((( t[0], t[1]), (t[2], t[3])), ((t[4], t[5]), (t[6], t[7])))
    inv = s256_inv(c, a, N, V)
    ib = [inv[0][0][0], inv[0][0][1], inv[0][1][0], inv[0][1][1],
          inv[1][0][0], inv[1][0][1], inv[1][1][0], inv[1][1][1]]
    # out = A Minv ib + 0x63 ; A as the AES affine matrix
    AM = []
    for i in range(8):
        col = Minv[i]  # tower bit i -> AES-basis value col
        # affine (no constant) of col
        s = 0
        for k in range(8):
            bit = ((col >> k) ^ (col >> ((k + 4) % 8)) ^ (col >> ((k + 5) % 8)) ^
                   (col >> ((k + 6) % 8)) ^ (col >> ((k + 7) % 8))) & 1
            s |= bit << k
        AM.append(s)
    out = [frozenset()] * 8
    for i in range(8):
        for k in range(8):
            if AM[i] >> k & 1:
                out[k] = X(out[k], ib[i])
    return c, out


def evaluate(c, out, v):
    sig = {i: (v >> i) & 1 for i in range(8)}
    for k, (a, b) in enumerate(c.ands):
        sig[8 + k] = (sum(sig[s] for s in a) & 1) & (sum(sig[s] for s in b) & 1)
    r = 0
    for k in range(8):
        r |= (sum(sig[s] for s in out[k]) & 1) << k
    return r ^ 0x63


def paar(targets, first_new):
    """Greedy common-pair elimination over a list of XOR sets; returns (gates, rewritten targets)."""
    targets = [set(t) for t in targets]
    gates = []
    nxt = first_new
    while True:
        count = {}
        for t in targets:
            if len(t) < 2:
                continue
            for p in itertools.combinations(sorted(t), 2):
                count[p] = count.get(p, 0) + 1
        if not count:
            break
        p, n = max(count.items(), key=lambda kv: (kv[1], -kv[0][0], -kv[0][1]))
        if n < 2:
            # no sharing left: build each remaining set as a chain
            for t in targets:
                while len(t) >= 2:
                    a, b = sorted(t)[:2]
                    gates.append(('x', nxt, a, b))
                    t -= {a, b}
                    t.add(nxt)
                    nxt += 1
            break
        gates.append(('x', nxt, p[0], p[1]))
        for t in targets:
            if p[0] in t and p[1] in t:
                t -= set(p)
                t.add(nxt)
        nxt += 1
    return gates, [next(iter(t)) if t else None for t in targets], nxt


def emit(c, out):
    """C statements over u32 planes: inputs x0..x7 (bit 0 = LSB), outputs y0..y7.  Every linear
    target (the two inputs of each AND, the 8 outputs) is reduced by Paar's greedy pair
    elimination over all targets at once; the gates are then emitted in dependency order."""
    targets = [set(a) for a, _ in c.ands] + [set(b) for _, b in c.ands] + [set(o) for o in out]
    gates, roots, _ = paar(targets, 1000)
    na = len(c.ands)
    xor_of = {g[1]: (g[2], g[3]) for g in gates}
    and_in = {8 + k: (roots[k], roots[na + k]) for k in range(na)}
    names, lines, done = {}, [], set()

    def name(sgn):
        if sgn is None:
            return '0u'
        if sgn < 8:
            return f'x{sgn}'
        return names[sgn]

    def visit(sgn):
        if sgn is None or sgn < 8 or sgn in done:
            return
        done.add(sgn)
        if sgn in xor_of:
            a, b = xor_of[sgn]
            visit(a)
            visit(b)
            names[sgn] = f't{sgn}'
            lines.append(f'const uint32_t t{sgn} = {name(a)} ^ {name(b)};')
        else:
            a, b = and_in[sgn]
            visit(a)
            visit(b)
            names[sgn] = f'm{sgn}'
            lines.append(f'const uint32_t m{sgn} = {name(a)} & {name(b)};')

    for k in range(8):
        visit(roots[2 * na + k])
    for k in range(8):  # outputs into temporaries first: y may alias x (an in-place S-box)
        inv = '~' if (0x63 >> k) & 1 else ''
        lines.append(f'const uint32_t o{k} = {inv}{name(roots[2 * na + k])};')
    for k in range(8):
        lines.append(f'y{k} = o{k};')
    n_xor = sum(1 for ln in lines if ' ^ ' in ln)
    n_and = sum(1 for ln in lines if ' & ' in ln)
    return lines, n_xor, n_and


def evaluate_lines(lines, v):
    env = {f'x{i}': (v >> i) & 1 for i in range(8)}
    for ln in lines:
        ln = ln.replace('const uint32_t ', '').rstrip(';')
        lhs, rhs = [x.strip() for x in ln.split('=')]
        rhs = rhs.replace('~', '1 ^ ').replace('0u', '0')
        env[lhs] = eval(rhs, {}, env) & 1
    env.update({f'y{k}': env[f'o{k}'] for k in range(8)})
    return sum(env[f'y{k}'] << k for k in range(8))


def main():
    c, out = build()
    tab = sbox_table()
    bad = [v for v in range(256) if evaluate(c, out, v) != tab[v]]
    assert not bad, bad[:8]
    lines, n_xor, n_and = emit(c, out)
    bad = [v for v in range(256) if evaluate_lines(lines, v) != tab[v]]
    assert not bad, ('emitted circuit', bad[:8])
    print('// generated by scripts/ubench/sbox_circuit.py -- bitsliced AES S-box, tower field')
    print(f'// {n_and} AND + {n_xor} XOR (2-input; the compiler fuses XOR pairs into v_bitop3_b32)')
    print('#define AES_SBOX_BITSLICED(x0, x1, x2, x3, x4, x5, x6, x7, y0, y1, y2, y3, y4, y5, y6, y7) \\')
    print('    do { \\')
    for ln in lines:
        print('        ' + ln + ' \\')
    print('    } while (0)')
    print(f'checked all 256 inputs: {n_and} AND, {n_xor} XOR', file=sys.stderr)


if __name__ == '__main__':
    main()

"""Surface-probe recipe shared by make_golden.py (reference) and tests/test_surface.py."""
SURFACE_CASES = [
    # (name, ctor args as JSON-able description, call)
    ('ctor_ok', ['int:1', 'int:10', 'bytes:ff*16'], None),
    ('ctor_kw', 'kw', None),
    ('ctor_neg', ['int:-1', 'int:10', 'bytes:ff*16'], None),
    ('ctor_float', ['float:1.0', 'int:10', 'bytes:ff*16'], None),
    ('ctor_bool', ['bool:1', 'int:10', 'bytes:ff*16'], None),
    ('ctor_big', ['int:18446744073709551616', 'int:10', 'bytes:ff*16'], None),
    ('ctor_max_u64', ['int:1', 'int:18446744073709551615', 'bytes:ff*16'], None),
    ('ctor_str_key', ['int:1', 'int:10', 'str:x*16'], None),
    ('ctor_list_key', ['int:1', 'int:10', 'list:255*16'], None),
    ('ctor_bytearray_key', ['int:1', 'int:10', 'bytearray:ff*16'], None),
    ('ctor_memoryview_key', ['int:1', 'int:10', 'memoryview:ff*16'], None),
    ('ctor_key15', ['int:1', 'int:10', 'bytes:ff*15'], None),
    ('ctor_key17', ['int:1', 'int:10', 'bytes:ff*17'], None),
    ('ctor_u32x4_key', ['int:1', 'int:10', 'u32:4'], None),
    ('ctor_min_gt_max', ['int:11', 'int:10', 'bytes:ff*16'], None),
    ('ctor_order', ['int:11', 'int:10', 'bytes:ff*3'], None),
    ('ctor_bad_key', ['int:1', 'int:10', 'bytes:00*8+ff*8'], None),
    ('ctor_two_args', ['int:1', 'int:10'], None),
    ('set_min', ['int:5', 'int:10', 'bytes:ff*16'], 'set_min'),
    ('next_no_final', ['int:5', 'int:10', 'bytes:ff*16'], 'next_no_final'),
    ('next_kw', ['int:5', 'int:10', 'bytes:ff*16'], 'next_kw'),
    ('next_int_final', ['int:5', 'int:10', 'bytes:ff*16'], 'next_int_final'),
    ('next_none_final', ['int:5', 'int:10', 'bytes:ff*16'], 'next_none_final'),
    ('next_str_final', ['int:5', 'int:10', 'bytes:ff*16'], 'next_str_final'),
    ('next_str_buf', ['int:5', 'int:10', 'bytes:ff*16'], 'next_str_buf'),
    ('next_bytearray', ['int:5', 'int:10', 'bytes:ff*16'], 'next_bytearray'),
    ('next_u32_items', ['int:5', 'int:10', 'bytes:ff*16'], 'next_u32_items'),
]


def surface_value(desc):
    kind, _, v = desc.partition(':')
    if kind == 'int':
        return int(v)
    if kind == 'float':
        return float(v)
    if kind == 'bool':
        return bool(int(v))
    if kind in ('bytes', 'bytearray', 'memoryview'):
        out = b''
        for part in v.split('+'):
            byte, n = part.split('*')
            out += bytes([int(byte, 16)]) * int(n)
        return {'bytes': bytes, 'bytearray': bytearray, 'memoryview': memoryview}[kind](out)
    if kind == 'str':
        ch, n = v.split('*')
        return ch * int(n)
    if kind == 'list':
        x, n = v.split('*')
        return [int(x)] * int(n)
    if kind == 'u32':
        import numpy as np
        return np.full(int(v), 0xFFFFFFFF, np.uint32)
    raise ValueError(desc)


def surface_call(mod, args, call):
    C = mod._gclmulchunker
    if args == 'kw':
        return C(min_length=1, max_length=10, key=b'\xff' * 16)
    c = C(*[surface_value(a) for a in args])
    if call is None:
        return (c.min_length, c.max_length)
    if call == 'set_min':
        c.min_length = 3
    data = b'\xaa' * 30
    import numpy as np
    return {
        'next_no_final': lambda: c.next_cut(data),
        'next_kw': lambda: c.next_cut(data, final=True),
        'next_int_final': lambda: c.next_cut(data, 1),
        'next_none_final': lambda: c.next_cut(data, None),
        'next_str_final': lambda: c.next_cut(data, 'yes'),
        'next_str_buf': lambda: c.next_cut('a' * 30, True),
        'next_bytearray': lambda: c.next_cut(bytearray(data), False),
        'next_u32_items': lambda: c.next_cut(np.full(8, 0xAAAAAAAA, np.uint32), True),
    }.get(call, lambda: None)()



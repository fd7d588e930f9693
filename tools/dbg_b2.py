import hashlib, numpy as np, sys
sys.path.insert(0, '.')
import mysticeti_amd as M
with M.Engine(devices=(0,)) as e:
    for lens in ([0, 1, 5, 64, 127, 128, 129, 200, 256, 257, 1000], list(range(40))):
        items = [bytes((i * 31 + 7) % 251 for i in range(n)) for n in lens]
        out = e.blake2b256(items)
        for it, o in zip(items, out):
            ok = bytes(o) == hashlib.blake2b(it, digest_size=32).digest()
            print(len(it), ok, bytes(o).hex()[:32], hashlib.blake2b(it, digest_size=32).hexdigest()[:32])

def jit(*a, **k):
    if a and callable(a[0]) and len(a) == 1 and not k:
        return a[0]
    return lambda f: f
njit = jit
prange = range

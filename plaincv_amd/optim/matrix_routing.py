"""Shared routing for matrix preconditioners (mirrors optim/matrix_routing.py:8-40).

Leaves are identified by their Flax path string ("a/b/kernel"), exactly the
string ``path_to_name`` builds in the reference, so routing decisions are the
reference's.
"""


def path_to_name(path) -> str:
    if isinstance(path, str):
        return path
    parts = []
    for key in path:
        for attr in ("key", "name", "idx"):
            if hasattr(key, attr):
                parts.append(str(getattr(key, attr)))
                break
        else:
            parts.append(str(key))
    return "/".join(parts)


def is_non_degenerate_2d_matrix(p) -> bool:
    shape = tuple(p.shape)
    return len(shape) == 2 and shape[0] > 1 and shape[1] > 1


def should_use_matrix_preconditioner(path, p) -> bool:
    """optim/matrix_routing.py:27-40: 2-D, both dims > 1, leaf 'kernel', and not an
    embedding / lm_head / norm parameter."""
    if not is_non_degenerate_2d_matrix(p):
        return False
    name = path_to_name(path).lower()
    leaf = name.split("/")[-1] if name else ""
    if leaf != "kernel":
        return False
    if ("embed" in name) or ("embedding" in name) or ("lm_head" in name):
        return False
    if "norm" in name:
        return False
    return True

"""Eager equivalents of jax.lax control flow (test infrastructure only)."""


def while_loop(cond_fun, body_fun, init_val):
    val = init_val
    while bool(cond_fun(val)):
        val = body_fun(val)
    return val


def cond(pred, true_fun, false_fun, *operands):
    if bool(pred):
        return true_fun(*operands)
    return false_fun(*operands)

"""BatchNorm (+ fused SnakeActivation) and standalone Snake on the HIP path."""
import torch

from ._native import call, grad_sink, ptr, stream_ptr, value


def _dims(x):
    B, C = x.shape[0], x.shape[1]
    return B, C, x.numel() // (B * C)


class _BNSnakeTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, a, running_mean, running_var, nbt, momentum, eps):
        ctx.params = (w, b, a)
        a = a.reshape(-1) if a is not None else None
        x = x.contiguous()
        B, C, HW = _dims(x)
        dev = x.device
        y = torch.empty_like(x)
        save = torch.empty(4 * C, device=dev, dtype=torch.float32)  # mean | invstd | scale | shift
        ws = torch.empty(value("tvq_bn_workspace", B, C, HW), device=dev, dtype=torch.uint8)
        call("tvq_bn_train_fwd", ptr(x), B, C, HW, ptr(w), ptr(b), ptr(running_mean),
             ptr(running_var), ptr(nbt), float(momentum), float(eps), ptr(a), ptr(y),
             ptr(save[:C]), ptr(save[C:2 * C]), ptr(save[2 * C:]), ptr(ws), stream_ptr())
        ctx.save_for_backward(x, w, a, save)
        ctx.has = (w is not None, b is not None, a is not None)
        return y

    @staticmethod
    def backward(ctx, gy):
        return _bn_snake_bwd(ctx, gy)


class _BNSnakeTrainPart(torch.autograd.Function):
    """The training BatchNorm (+ Snake) forward from the producing conv's per-block statistics
    (hip.conv.conv2d_bnstats: tvq_bn_train_apply_part, one launch); backward = _BNSnakeTrain's."""

    @staticmethod
    def forward(ctx, x, part, w, b, a, running_mean, running_var, nbt, momentum, eps):
        ctx.params = (w, b, a)
        a = a.reshape(-1) if a is not None else None
        x = x.contiguous()
        B, C, HW = _dims(x)
        y = torch.empty_like(x)
        save = torch.empty(4 * C, device=x.device, dtype=torch.float32)
        call("tvq_bn_train_apply_part", ptr(x), B, C, HW, ptr(part), part.shape[1], ptr(w), ptr(b),
             ptr(running_mean), ptr(running_var), ptr(nbt), float(momentum), float(eps), ptr(a),
             ptr(y), ptr(save[:C]), ptr(save[C:2 * C]), ptr(save[2 * C:]), stream_ptr())
        ctx.save_for_backward(x, w, a, save)
        ctx.has = (w is not None, b is not None, a is not None)
        return y

    @staticmethod
    def backward(ctx, gy):
        dx, dw, db, da = _bn_snake_bwd(ctx, gy)[:4]
        return dx, None, dw, db, da, None, None, None, None, None


def bn_snake_part(x, part, bn, a=None):
    """snake_a(BatchNorm_train(x)) with the statistics the conv that produced x wrote
    (hip.conv.conv2d_bnstats / conv_transpose2d_bnstats)."""
    if bn.momentum is None:
        raise NotImplementedError("cumulative-average BatchNorm (momentum=None) is not on the path")
    return _BNSnakeTrainPart.apply(x, part, bn.weight, bn.bias, a, bn.running_mean,
                                   bn.running_var, bn.num_batches_tracked, bn.momentum, bn.eps)


def _bn_snake_bwd(ctx, gy):
    """Backward of the training BatchNorm (+ Snake) (tvq_bn_bwd), shared by both forwards."""
    x, w, a, save = ctx.saved_tensors
    B, C, HW = _dims(x)
    dev = x.device
    g = gy.contiguous()
    dx = torch.empty_like(x)
    has_w, has_b, has_a = ctx.has
    sinks = [grad_sink(p) if h else None for p, h in zip(ctx.params, ctx.has)]
    direct = all((s is not None) == h for s, h in zip(sinks, ctx.has))
    if direct:
        dw, db, da = sinks
    else:
        dw = torch.empty(C, device=dev) if has_w else None
        db = torch.empty(C, device=dev) if has_b else None
        da = torch.empty(C, device=dev) if has_a else None
    ws = torch.empty(value("tvq_bn_workspace", B, C, HW), device=dev, dtype=torch.uint8)
    call("tvq_bn_bwd", ptr(g), ptr(x), B, C, HW, ptr(w), ptr(a), ptr(save[:C]),
         ptr(save[C:2 * C]), ptr(save[2 * C:]), ptr(dx), ptr(dw), ptr(db), ptr(da), int(direct),
         ptr(ws), stream_ptr())
    if direct:
        return dx, None, None, None, None, None, None, None, None
    if da is not None:
        da = da.view_as(ctx.params[2])
    return dx, dw, db, da, None, None, None, None, None


def bn_snake(x, bn, a=None):
    """snake_a(BatchNorm(x)) with the module `bn`'s parameters/buffers; a: the Snake
    parameter ((1,C,1,1) or (C,)) or None."""
    if bn.training:
        if bn.momentum is None:
            raise NotImplementedError("cumulative-average BatchNorm (momentum=None) is not on the path")
        return _BNSnakeTrain.apply(x, bn.weight, bn.bias, a, bn.running_mean, bn.running_var,
                                   bn.num_batches_tracked, bn.momentum, bn.eps)
    if torch.is_grad_enabled() and (x.requires_grad or (bn.weight is not None and bn.weight.requires_grad)):
        raise NotImplementedError("eval-mode BatchNorm backward is not on the TimeVQVAE path")
    x = x.contiguous()
    B, C, HW = _dims(x)
    y = torch.empty_like(x)
    ss = torch.empty(2 * C, device=x.device, dtype=torch.float32)
    a = a.reshape(-1) if a is not None else None
    call("tvq_bn_eval_fwd", ptr(x), B, C, HW, ptr(bn.weight), ptr(bn.bias), ptr(bn.running_mean),
         ptr(bn.running_var), float(bn.eps), ptr(a), ptr(y), ptr(ss), stream_ptr())
    return y


class _Snake(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, a):
        ctx.a_param = a
        a = a.reshape(-1)
        x = x.contiguous()
        B, C, HW = _dims(x)
        y = torch.empty_like(x)
        call("tvq_snake_fwd", ptr(x), B, C, HW, ptr(a), ptr(y), stream_ptr())
        ctx.save_for_backward(x, a)
        return y

    @staticmethod
    def backward(ctx, gy):
        return _snake_bwd(ctx, gy, None)


def _snake_bwd(ctx, gy, g_add):
    x, a = ctx.saved_tensors
    B, C, HW = _dims(x)
    g = gy.contiguous()
    if g_add is not None and (g_add.shape != x.shape or not g_add.is_contiguous()):
        g_add = g_add.contiguous().view_as(x)
    dx = torch.empty_like(x)
    sink = grad_sink(ctx.a_param)
    da = sink if sink is not None else torch.empty(C, device=x.device)
    ws = torch.empty(value("tvq_snake_workspace", B, C, HW), device=x.device, dtype=torch.uint8)
    call("tvq_snake_bwd", ptr(g), ptr(x), B, C, HW, ptr(a), ptr(g_add), ptr(dx), ptr(da),
         int(sink is not None), ptr(ws), stream_ptr())
    return dx, (None if sink is not None else da.view_as(ctx.a_param))


class _SnakeSkip(torch.autograd.Function):
    """(Snake(x), x): the second output is x itself for the ResBlock skip path, so the
    backward receives both gradients of x and sums them in the Snake backward kernel
    instead of autograd adding them in a separate launch."""

    @staticmethod
    def forward(ctx, x, a):
        y = _Snake.forward(ctx, x, a)
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, gy, gx):
        if gy is None:
            return gx, None
        return _snake_bwd(ctx, gy, gx)


def snake(x, a):
    """SnakeActivation (train_utils.py:446-448): x + (1/a) sin(a x)^2; a: the (1,C,1,1)
    parameter or a (C,) tensor."""
    return _Snake.apply(x, a)


def snake_skip(x, a):
    """(snake(x, a), x) with the two gradients of x summed inside the Snake backward."""
    return _SnakeSkip.apply(x, a)

"""Optimizer factories of spotlight/optimizers.py (reference :4-22), same names,
defaults and return types.  ImplicitFactorizationModel calls the factory it is
given on a probe parameter and reads the optimizer's kind and hyper-parameters
(``describe``); the update itself runs in the fused kernel."""
import torch
import torch.optim as optim


def sgd_optimizer(model_params, lr=1e-2, weight_decay=1e-6):
    return optim.SGD(model_params, lr=lr, weight_decay=weight_decay)


def adam_optimizer(model_params, lr=1e-2, betas=(0.5, 0.999), weight_decay=1e-6):
    return optim.Adam(model_params, lr=lr, betas=betas, weight_decay=weight_decay)


def rms_optimizer(model_params, lr=1e-2, weight_decay=0):
    return optim.RMSprop(model_params, lr=lr, weight_decay=weight_decay)


def describe(optimizer_func, lr, weight_decay):
    """Kind and hyper-parameters of the torch optimizer ``optimizer_func`` builds
    (called as implicit.py:182-192 calls it).  Raises NotImplementedError for a
    configuration the fused update does not implement."""
    probe = torch.nn.Parameter(torch.zeros(1))
    if optimizer_func is None:
        opt = optim.Adam([probe], weight_decay=weight_decay, lr=lr)       # implicit.py:182-187
    else:
        opt = optimizer_func([probe], weight_decay=weight_decay, lr=lr)
    g = opt.param_groups[0]
    d = dict(lr=float(g["lr"]), weight_decay=float(g.get("weight_decay", 0.0)))
    if type(opt) is optim.Adam:
        if g.get("amsgrad") or g.get("maximize") or g.get("decoupled_weight_decay", False):
            raise NotImplementedError("Adam variant (amsgrad/maximize/decoupled) not supported by the fused update")
        d.update(kind="adam", betas=tuple(float(b) for b in g["betas"]), eps=float(g["eps"]))
    elif type(opt) is optim.SGD:
        if g.get("momentum", 0) or g.get("nesterov") or g.get("dampening", 0) or g.get("maximize"):
            raise NotImplementedError("SGD with momentum/nesterov/dampening not supported by the fused update")
        d.update(kind="sgd")
    elif type(opt) is optim.RMSprop:
        if g.get("momentum", 0) or g.get("centered") or g.get("maximize"):
            raise NotImplementedError("RMSprop with momentum/centered not supported by the fused update")
        d.update(kind="rms", alpha=float(g["alpha"]), eps=float(g["eps"]))
    else:
        raise NotImplementedError(f"optimizer {type(opt).__name__} not supported by the fused update")
    return d

"""Parity verdicts of the full-size GPU tests, with the elementwise numbers reported.

`check` applies oracle.mf.tensor_parity (the norm rule) and oracle.mf.elementwise_parity
(every element within 1e-5 of the fp32 reference or inside the fp64 band) and reports the
elementwise figures two ways: a ParityReport warning (pytest lists it in the warnings
summary of the run's log, -q included) and a JSON line appended to
gpurun_out/parity_elementwise.jsonl (kept under profiles/ per round)."""
import json
import os
import warnings

from oracle import mf as omf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class ParityReport(UserWarning):
    pass


def order_stats(got, ref32, order32, rtol=1e-5):
    """The reference's own fp32 spread on the elements the GPU leaves outside rtol: ``order32`` is
    a second fp32 restatement of the same steps summing the gradients in another order
    (MFOracle(order_seed=...)).  Returns n_ref_out (elements where the two fp32 restatements
    differ beyond rtol), n_gpu_out, n_both (GPU outside AND the second order outside too on the
    same element) and max_ref_rel (max |order32 - ref32| / max |ref32|)."""
    import torch
    g = torch.as_tensor(got).double().reshape(-1).cpu()
    r = torch.as_tensor(ref32).double().reshape(-1)
    a = torch.as_tensor(order32).double().reshape(-1)
    mx = float(r.abs().max()) if r.numel() else 0.0
    tol = rtol * r.abs() + rtol * 1e-3 * mx
    gout = (g - r).abs() > tol
    aout = (a - r).abs() > tol
    return {"n_ref_out": int(aout.sum()), "n_gpu_out": int(gout.sum()), "n_both": int((gout & aout).sum()),
            "max_ref_rel": float((a - r).abs().max()) / max(mx, 1e-30) if r.numel() else 0.0}


def check(tag, got, ref32, ref64=None, before=None, rtol=1e-5, band=3.0, noise=None, alt32=None, order32=None,
          elementwise=True, kink=None):
    """``elementwise`` False: the verdict is the norm rule's alone, the elementwise figures are
    reported (a free-running trajectory past the depth where equally valid fp32 orders part
    element by element, tests/test_configs_gpu.py NCF_STEPS)."""
    ok_n, msg = omf.tensor_parity(got, ref32, ref64, rtol=rtol, band=band, before=before, alt32=alt32)
    ok_e, st = omf.elementwise_parity(got, ref32, ref64, rtol=rtol, band=band, before=before, noise=noise,
                                      alt32=alt32, kink=kink)
    line = (f"{tag}{'' if elementwise else ' (reported)'}: max|d|/max|ref| {st['max_rel']:.2e}, "
            f"outside 1e-5 {st['n_out']}/{st['n']} ({st['frac_out']:.2e}), ill-conditioned {st['n_ill']}, failing the fp64 band too {st['n_fail']}")
    if order32 is not None:
        st["order"] = order_stats(got, ref32, order32, rtol)
        o = st["order"]
        line += (f"; the reference in another fp32 summation order: outside 1e-5 on {o['n_ref_out']} elements, "
                 f"{o['n_both']} of the GPU's {o['n_gpu_out']} among them")
    warnings.warn(line, ParityReport)
    try:
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", "parity_elementwise.jsonl"), "a") as f:
            f.write(json.dumps({"tag": tag, "norm_ok": ok_n, "norm": msg, "elementwise_asserted": elementwise,
                                **st}) + "\n")
    except OSError:
        pass
    return ok_n and (ok_e or not elementwise), f"{msg}; {line}"

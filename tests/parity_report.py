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


def check(tag, got, ref32, ref64=None, before=None, rtol=1e-5, band=3.0, noise=None, alt32=None):
    ok_n, msg = omf.tensor_parity(got, ref32, ref64, rtol=rtol, band=band, before=before)
    ok_e, st = omf.elementwise_parity(got, ref32, ref64, rtol=rtol, band=band, before=before, noise=noise,
                                      alt32=alt32)
    line = (f"{tag}: max|d|/max|ref| {st['max_rel']:.2e}, outside 1e-5 {st['n_out']}/{st['n']} "
            f"({st['frac_out']:.2e}), ill-conditioned {st['n_ill']}, failing the fp64 band too {st['n_fail']}")
    warnings.warn(line, ParityReport)
    try:
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", "parity_elementwise.jsonl"), "a") as f:
            f.write(json.dumps({"tag": tag, "norm_ok": ok_n, "norm": msg, **st}) + "\n")
    except OSError:
        pass
    return ok_n and ok_e, f"{msg}; {line}"

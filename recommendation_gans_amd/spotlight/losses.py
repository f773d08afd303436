"""Loss functions of the implicit-feedback models -- the reference's loss extension point
(spotlight/losses.py:20-172; chosen by name in implicit.py:194-199).

Signature ``loss(positive_predictions, negative_predictions=None, mask=None) -> 0-d tensor``
on PREDICTIONS (BilinearNet / MLP outputs are already sigmoided, representations.py:91).
These are plain tensor expressions for callers that score pairs themselves (a custom
``representation``'s outputs, ``ImplicitFactorizationModel._loss_func``).  The fused
training step does not call them: librg_hip.so computes the same four losses inside
``mf_pairs_kernel`` / ``ncf_pairs_kernel`` (include/rg_hip.h RG_LOSS_*), and
``tests/test_losses_cpu.py`` pins these functions against the reference's golden steps.

Semantics kept from the reference, including its quirks:
* ``pointwise_loss``: BCE mean over the positives (target 1) plus BCE mean over the
  negatives (target 0), each log clamped at -100 as nn.BCELoss; with ``mask`` the scalar
  loss is multiplied by the mask and renormalised (:52-55), i.e. it returns the loss;
* ``bpr_loss``: mean(1 - sigmoid(pos - neg)) on the predictions, broadcast as given (the
  reference's live shapes pos (B,) / neg (n*B,) raise; the fused step's
  'pairwise_bpr' pairs ``neg.view(n, B)`` against ``pos``, which is what passing
  ``negative_predictions.view(n, -1)`` here computes);
* ``hinge_loss``: mean(clamp(neg - pos + 1, 0));
* ``adaptive_hinge_loss``: the hinge against ``max(negative_predictions, 0)`` -- with the
  live flat negatives the single global maximum.
``ratio`` is accepted and unused, as in the reference.
"""
import torch

__all__ = ["pointwise_loss", "bpr_loss", "hinge_loss", "adaptive_hinge_loss", "LOSS_FUNCTIONS", "loss_for"]


def _bce_mean(p, target):
    # nn.BCELoss (mean): -(t*log(p) + (1-t)*log(1-p)), each log clamped at -100
    if target == 1:
        return -torch.clamp(torch.log(p), min=-100.0).mean()
    return -torch.clamp(torch.log(1.0 - p), min=-100.0).mean()


def _masked(loss, mask):
    if mask is None:
        return loss.mean()
    mask = mask.float()
    loss = loss * mask
    return loss.sum() / mask.sum()


def pointwise_loss(positive_predictions, negative_predictions=None, mask=None):
    """Logistic loss (spotlight/losses.py:20-56)."""
    loss = _bce_mean(positive_predictions, 1)
    if negative_predictions is not None:
        loss = loss + _bce_mean(negative_predictions, 0)
    if mask is not None:
        mask = mask.float()
        loss = loss * mask
        return loss.sum() / mask.sum()
    return loss


def bpr_loss(positive_predictions, negative_predictions, mask=None, ratio=1):
    """BPR pairwise loss (spotlight/losses.py:59-96)."""
    return _masked(1.0 - torch.sigmoid(positive_predictions - negative_predictions), mask)


def hinge_loss(positive_predictions, negative_predictions, mask=None, ratio=1):
    """Hinge pairwise loss (spotlight/losses.py:99-130)."""
    return _masked(torch.clamp(negative_predictions - positive_predictions + 1.0, 0.0), mask)


def adaptive_hinge_loss(positive_predictions, negative_predictions, mask=None, ratio=1):
    """Hinge against the highest negative over dim 0 (spotlight/losses.py:133-172)."""
    highest, _ = torch.max(negative_predictions, 0)
    return hinge_loss(positive_predictions, highest.squeeze(), mask=mask)


LOSS_FUNCTIONS = {"pointwise": pointwise_loss, "bpr": bpr_loss, "hinge": hinge_loss,
                  "adaptive_hinge": adaptive_hinge_loss}


def loss_for(name):
    """The function the reference's ImplicitFactorizationModel selects for a loss name
    (implicit.py:194-199): 'pointwise', 'hinge', anything else -> adaptive hinge."""
    if name == "pointwise":
        return pointwise_loss
    if name == "hinge":
        return hinge_loss
    return adaptive_hinge_loss

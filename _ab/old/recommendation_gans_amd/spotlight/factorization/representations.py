"""BilinearNet (spotlight/factorization/representations.py:16-91, reference).

The module holds the four tables with the reference's parameter names and
initialisation (state_dict keys ``user_embeddings.weight``, ``item_embeddings.weight``,
``user_biases.weight``, ``item_biases.weight`` -- the checkpoint format of
implicit.py:467-471).  Its forward, sigmoid(<u, i> + b_u + b_i), runs on the GPU
through rg_mf_scores; training never calls it (the fused step does)."""
import torch
import torch.nn as nn

from ..layers import ScaledEmbedding, ZeroEmbedding


class BilinearNet(nn.Module):
    def __init__(self, num_users, num_items, embedding_dim=32, user_embedding_layer=None,
                 item_embedding_layer=None, sparse=False):
        super().__init__()
        self.embedding_dim = embedding_dim
        self.user_embeddings = user_embedding_layer or ScaledEmbedding(num_users, embedding_dim, sparse=sparse)
        self.item_embeddings = item_embedding_layer or ScaledEmbedding(num_items, embedding_dim, sparse=sparse)
        self.user_biases = ZeroEmbedding(num_users, 1, sparse=sparse)
        self.item_biases = ZeroEmbedding(num_items, 1, sparse=sparse)

    def forward(self, user_ids, item_ids):
        from ... import _lib
        from ..._lib import check, ptr
        if not self.user_embeddings.weight.is_cuda:
            raise RuntimeError("BilinearNet.forward runs on the GPU (librg_hip.so); move the module to cuda")
        lib = _lib.load()
        u = user_ids.reshape(-1).to(torch.int64).contiguous()
        i = item_ids.reshape(-1).to(torch.int64).contiguous()
        if u.numel() != i.numel():
            u, i = torch.broadcast_tensors(u, i)
            u, i = u.contiguous(), i.contiguous()
        out = torch.empty(u.numel(), dtype=torch.float32, device=u.device)
        w = [self.user_embeddings.weight, self.item_embeddings.weight, self.user_biases.weight,
             self.item_biases.weight]
        w = [t.detach().float().contiguous() for t in w]
        check(lib.rg_mf_scores(_lib.stream_handle(), ptr(w[0]), ptr(w[1]), ptr(w[2]), ptr(w[3]), self.embedding_dim,
                               ptr(u), ptr(i), u.numel(), ptr(out)), "rg_mf_scores")
        return out

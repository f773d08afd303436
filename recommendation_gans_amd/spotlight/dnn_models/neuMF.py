"""NeuMF (spotlight/dnn_models/neuMF.py:7-62 of the reference).

Same constructor, parameter names (``embedding_user_mlp.weight``,
``embedding_item_mlp.weight``, ``embedding_user_mf.weight``,
``embedding_item_mf.weight``, ``layers.{3k}.weight/bias``,
``affine_output.weight/bias``) and initialisation (nn.Embedding's N(0, 1);
Xavier-uniform Linear weights, biases 0.01, applied in module order), so a torch
seed gives the reference's tensors.  Training runs through the fused NCF step with
the GMF branch (ncf_engine, rg_ncf_pairs with mf_dim = M, rg_neumf_apply);
``forward`` is the eval-mode scorer on the device."""
import torch
import torch.nn as nn


class NeuMF(nn.Module):
    def __init__(self, mlp_layers, num_users, num_items, mf_embedding_dim=25, mlp_embedding_dim=32):
        super().__init__()
        self.num_users, self.num_items = num_users, num_items
        self.latent_dim_mf, self.latent_dim_mlp = mf_embedding_dim, mlp_embedding_dim
        self.embedding_user_mlp = nn.Embedding(num_embeddings=num_users, embedding_dim=mlp_embedding_dim)
        self.embedding_item_mlp = nn.Embedding(num_embeddings=num_items, embedding_dim=mlp_embedding_dim)
        self.embedding_user_mf = nn.Embedding(num_embeddings=num_users, embedding_dim=mf_embedding_dim)
        self.embedding_item_mf = nn.Embedding(num_embeddings=num_items, embedding_dim=mf_embedding_dim)
        self.layers = nn.ModuleList()
        for idx in range(len(mlp_layers) - 1):
            self.layers.append(nn.Linear(mlp_layers[idx], mlp_layers[idx + 1]))
            self.layers.append(nn.LeakyReLU(0.1, inplace=True))
            self.layers.append(nn.Dropout(0.5))
        self.affine_output = nn.Linear(mlp_layers[-1] + mf_embedding_dim, out_features=1)
        self.logistic = nn.Sigmoid()
        self.apply(self.init_weights)

    def linears(self):
        return [m for m in self.layers if isinstance(m, nn.Linear)] + [self.affine_output]

    def forward(self, user_indices, item_indices):
        if not self.embedding_user_mlp.weight.is_cuda:
            raise RuntimeError("NeuMF.forward runs on the GPU; move the module to cuda")
        x = torch.cat([self.embedding_user_mlp(user_indices), self.embedding_item_mlp(item_indices)], dim=-1)
        for m in self.layers:
            x = m(x)
        gmf = self.embedding_user_mf(user_indices) * self.embedding_item_mf(item_indices)
        return self.logistic(self.affine_output(torch.cat([x, gmf], dim=-1)))

    def init_weights(self, m):
        if type(m) == nn.Linear:
            torch.nn.init.xavier_uniform_(m.weight)
            m.bias.data.fill_(0.01)

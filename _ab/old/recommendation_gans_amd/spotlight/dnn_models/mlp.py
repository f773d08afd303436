"""NCF MLP (spotlight/dnn_models/mlp.py:5-46 of the reference).

Same constructor, parameter names (``embedding_user.weight``,
``embedding_item.weight``, ``layers.{3k}.weight/bias``, the output Linear last)
and initialisation (nn.Embedding's N(0, 1); Xavier-uniform Linear weights,
biases 0.01, applied in module order), so a checkpoint or a torch seed gives the
reference's tensors.  Training runs through the fused NCF step (ncf_engine);
``forward`` is the eval-mode scorer on the device."""
import torch
import torch.nn as nn


class MLP(nn.Module):
    def __init__(self, layers, num_users, num_items, output_dim=1, embedding_dim=32):
        super().__init__()
        self.num_users, self.num_items, self.latent_dim = num_users, num_items, embedding_dim
        self.embedding_user = nn.Embedding(num_embeddings=num_users, embedding_dim=embedding_dim)
        self.embedding_item = nn.Embedding(num_embeddings=num_items, embedding_dim=embedding_dim)
        self.layers = nn.ModuleList()
        for idx in range(len(layers) - 1):
            self.layers.append(nn.Linear(layers[idx], layers[idx + 1]))
            self.layers.append(nn.LeakyReLU(0.1, inplace=True))
            self.layers.append(nn.Dropout(0.5))
        self.layers.append(nn.Linear(layers[-1], out_features=1))
        self.logistic = nn.Sigmoid()
        self.apply(self.init_weights)

    def linears(self):
        return [m for m in self.layers if isinstance(m, nn.Linear)]

    def forward(self, user_indices, item_indices):
        if not self.embedding_user.weight.is_cuda:
            raise RuntimeError("MLP.forward runs on the GPU; move the module to cuda")
        x = torch.cat([self.embedding_user(user_indices), self.embedding_item(item_indices)], dim=-1)
        for m in self.layers[:-1]:
            x = m(x)
        return self.logistic(self.layers[-1](x))

    def init_weights(self, m):
        if type(m) == nn.Linear:
            torch.nn.init.xavier_uniform_(m.weight)
            m.bias.data.fill_(0.01)

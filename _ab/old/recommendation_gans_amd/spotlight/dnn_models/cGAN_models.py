"""cGAN generator / discriminator modules (spotlight/dnn_models/cGAN_models.py of the
reference).

Same constructors, submodule structure, parameter / buffer names and
initialisation order (nn.Embedding N(0, 1) with a zero padding row N, the layers'
default init, then Xavier-uniform Linear weights with biases 0.01 applied in
module order), so ``torch.manual_seed(s)`` followed by construction yields the
reference's tensors and checkpoints load either way.  Training runs through the
fused HIP iterations (recommendation_gans_amd.gan_engine via CGANs.CGAN); these
modules hold the parameters and give the plain forward on the GPU for callers that
use the networks directly."""
import torch
import torch.nn as nn


def _xavier_bias(m):
    if type(m) == nn.Linear:
        torch.nn.init.xavier_uniform_(m.weight)
        m.bias.data.fill_(0.01)


def _require_gpu(t):
    if not t.is_cuda:
        raise RuntimeError("cGAN modules run on the GPU; move the module to cuda")


class generator(nn.Module):
    """noise (B, noise_dim) + history ids (B, L) (padding = num_items) -> S tanh heads
    over the items, or (B, S) argmax slates with ``inference=True``."""

    def __init__(self, noise_dim=100, embedding_dim=50, hidden_layer=[16], num_items=1447, output_dim=3):
        super().__init__()
        self.z, self.y = noise_dim, embedding_dim
        self.num_items, self.output_dim = num_items, output_dim
        self.embedding_layer = nn.Embedding(num_items + 1, embedding_dim, padding_idx=num_items)
        widths = [noise_dim + embedding_dim] + list(hidden_layer)
        self.layers = nn.ModuleList()
        for a, b in zip(widths[:-1], widths[1:]):
            self.layers.extend([nn.Linear(a, b), nn.BatchNorm1d(num_features=b), nn.Dropout(0.1),
                                nn.LeakyReLU(0.2, inplace=True)])
        self.mult_heads = nn.ModuleDict({f"head_{s}": nn.Linear(widths[-1], num_items) for s in range(output_dim)})
        self.apply(self.init_weights)
        self.non_linear_emb = nn.LeakyReLU(0.2, inplace=True)

    def forward(self, noise, user_batch, inference=False):
        _require_gpu(noise)
        v = torch.cat([noise, self.embedding_layer(user_batch.long()).sum(1)], dim=1)
        v = self.non_linear_emb(v)
        for layer in self.layers:
            v = layer(v)
        heads = [torch.tanh(h(v)) for h in self.mult_heads.values()]
        if inference:
            return torch.stack([torch.max(h, 1)[1] for h in heads], 1).float().cpu()
        return tuple(heads)

    def init_weights(self, m):
        _xavier_bias(m)


class discriminator(nn.Module):
    """slate (B, S * num_items) one-hot or generated + history ids (B, L) -> (B, 1)."""

    def __init__(self, embedding_dim=50, hidden_layers=[16], input_dim=3, num_items=1447):
        super().__init__()
        self.non_linear_emb = nn.LeakyReLU(0.2, inplace=True)
        self.slate_size, self.user_condition, self.num_items = input_dim, embedding_dim, num_items
        self.embedding_layer = nn.Embedding(num_items + 1, embedding_dim, padding_idx=num_items)
        widths = [input_dim * num_items + embedding_dim] + list(hidden_layers) + [1]
        self.layers = nn.ModuleList()
        for a, b in zip(widths[:-2], widths[1:-1]):
            self.layers.extend([nn.Linear(a, b), nn.Dropout(0.3), nn.LeakyReLU(0.2)])
        self.layers.append(nn.Linear(widths[-2], widths[-1]))
        self.apply(self.init_weights)

    def forward(self, batch_input, condition):
        _require_gpu(batch_input)
        v = torch.cat([self.embedding_layer(condition.long()).sum(1), batch_input], dim=1).float()
        for layer in self.layers:
            v = layer(v)
        return v

    def init_weights(self, m):
        _xavier_bias(m)

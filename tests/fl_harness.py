"""The Flower client's quantization hook without flwr (config C5).

Restates what SImulation_Results_datasets/MNIST/Codes/Type_unbiased.py does around the
drop-in, so a test can run it unchanged with this package's quantizers:
  Net                    FLM:37-56   (the MNIST CNN; conv3/conv4 exist but forward skips them)
  local_train            FLM:69-83 + FLM:214-219 (SGD lr 0.1, momentum 0.9, one pass)
  HookClient.get_parameters   FLM:148-212 (flatten state_dict, delta vs the global model,
                         quantization_func(delta_tensor, bits), NMSE_info_<k>.pkl under
                         <nmse_dir>/<func.__name__>/rate_<bits>/, quantized delta + global
                         reshaped per layer)
flwr, Ray, torchvision and the MNIST files are absent here, so the data are synthetic
MNIST-shaped batches and the timing file (FLM:157-165) is left out."""
from __future__ import annotations

import os
import pickle

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


class Net(nn.Module):
    """FLM:37-56, layer for layer (172 554 parameters for 10 classes)."""

    def __init__(self, num_classes: int) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(1, 16, 5)
        self.pool = nn.MaxPool2d(2, 2)
        self.conv2 = nn.Conv2d(16, 32, 5)
        self.conv3 = nn.Conv2d(32, 64, 3)
        self.conv4 = nn.Conv2d(64, 128, 3)
        self.fc1 = nn.Linear(32 * 4 * 4, 128)
        self.dropout = nn.Dropout(0.5)
        self.fc2 = nn.Linear(128, num_classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.pool(F.relu(self.conv1(x)))
        x = self.pool(F.relu(self.conv2(x)))
        x = x.view(-1, 32 * 4 * 4)
        x = F.relu(self.fc1(x))
        x = self.dropout(x)
        return self.fc2(x)


def local_train(model: nn.Module, batches, lr: float = 0.1):
    """FLM:69-83 with FLM:217's optimizer, on CPU batches of (images, labels)."""
    crit = nn.CrossEntropyLoss()
    opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9)
    model.train()
    for images, labels in batches:
        opt.zero_grad()
        crit(model(images), labels).backward()
        opt.step()


def synthetic_batches(seed: int, n: int = 2, bs: int = 64):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(bs, 1, 28, 28, generator=g), torch.randint(0, 10, (bs,), generator=g)) for _ in range(n)]


class HookClient:
    """FlowerClient.get_parameters (FLM:148-212) around `quant_func`."""

    def __init__(self, model: nn.Module, quant_func, bits, nmse_dir: str, device="cuda"):
        self.model = model
        self.quantization_func = quant_func
        self.bits_per_dimension = bits
        self.nmse_dir = nmse_dir
        self.device = device
        self.global_model_params_np_array = np.zeros(sum(p.numel() for p in model.parameters() if p.requires_grad))
        self.last = {}

    def set_parameters(self, parameters):                         # FLM:141-146
        sd = {k: torch.Tensor(v) for k, v in zip(self.model.state_dict().keys(), parameters)}
        self.model.load_state_dict(sd, strict=True)
        self.global_model_params_np_array = np.concatenate([np.reshape(v.cpu().numpy(), -1) for v in sd.values()])

    def get_parameters(self):
        np_arrays = [val.cpu().numpy() for val in self.model.state_dict().values()]
        shapes = [np.shape(a) for a in np_arrays]
        sizes = np.array([np.size(a) for a in np_arrays])
        concat = np.concatenate([np.reshape(a, a.size) for a in np_arrays])
        gradient = concat - self.global_model_params_np_array     # f64 when the global is the f64 zeros
        gradient_tensor = torch.from_numpy(gradient).float().to(self.device)
        self.last["gradient"] = gradient_tensor.cpu().numpy()
        self.last["rng_before"] = torch.get_rng_state()
        out = self.quantization_func(gradient_tensor, self.bits_per_dimension)
        qt = torch.from_numpy(out).to(self.device) if isinstance(out, np.ndarray) else out
        err = qt - gradient_tensor
        gnorm = torch.norm(gradient_tensor).item()
        rate_dir = os.path.join(self.nmse_dir, self.quantization_func.__name__, f"rate_{self.bits_per_dimension}")
        os.makedirs(rate_dir, exist_ok=True)
        idx = sorted(int(f.split("_")[-1].split(".")[0]) for f in os.listdir(rate_dir)
                     if f.startswith("NMSE_info_") and f.endswith(".pkl"))
        nxt = max(idx) + 1 if idx else 1
        with open(os.path.join(rate_dir, f"NMSE_info_{nxt}.pkl"), "wb") as f:
            pickle.dump([err, gnorm], f)
        if isinstance(out, torch.Tensor):
            out = out.cpu().numpy()
        elif not isinstance(out, np.ndarray):
            raise TypeError("Quantization function must return a PyTorch tensor or a NumPy array.")
        self.last["quantized"] = out
        params = out + self.global_model_params_np_array
        layers = []
        for i, size in enumerate(sizes):
            lo = int(sizes[:i].sum())
            layers.append(params[lo:lo + size].reshape(shapes[i]))
        return layers

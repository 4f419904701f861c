"""Probe the host CPU's torch / numpy float arithmetic (is sqrt correctly rounded?)."""
import numpy as np, torch
x = torch.rand(1000000)*10+0.01
xd = x.double()
ref = np.sqrt(xd.numpy()).astype(np.float32)  # f64 sqrt rounded once
print("torch f32 sqrt mism", (torch.sqrt(x).numpy() != ref).sum())
print("numpy f32 sqrt mism", (np.sqrt(x.numpy()) != ref).sum())
print("torch f64 sqrt vs numpy f64 sqrt mism", (torch.sqrt(xd).numpy() != np.sqrt(xd.numpy())).sum())
print("torch f64->f32 sqrt mism", (torch.sqrt(xd).float().numpy() != ref).sum())
print("torch exp f64 vs numpy exp f64 mism", (torch.exp(xd/5).numpy() != np.exp(xd.numpy()/5)).sum(),
      "after f32 rounding", (torch.exp(xd/5).float().numpy() != np.exp(xd.numpy()/5).astype(np.float32)).sum())

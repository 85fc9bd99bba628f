import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from rafiki_amd.model.model import load_model_class
from rafiki_amd.models import model_file
clazz = load_model_class(open(model_file('FeedForward'), 'rb').read(), 'FeedForward')
m = clazz(epochs=3, hidden_layer_count=2, hidden_layer_units=128, learning_rate=0.001, batch_size=128, image_size=28)
m.train('synthetic://image?n=6000&size=28&channels=1&classes=10&seed=0')
print('eval graphed', m.evaluate('synthetic://image?n=1000&size=28&channels=1&classes=10&seed=1'))
imgs, labels, _ = m._load('synthetic://image?n=1000&size=28&channels=1&classes=10&seed=1')
eng = m._engine
x = eng.prepare_inputs(imgs)
p = eng.forward_eval(x)
print('eval eager', (p.argmax(1).cpu().numpy() == labels).mean())
_, logits = eng.reference_loss(x, None, training=False)
print('eval ref', (logits.argmax(1).cpu().numpy() == labels).mean())
print('running', eng.running[:, :5])
# train-mode accuracy on the train set
imgs2, labels2, _ = m._load('synthetic://image?n=6000&size=28&channels=1&classes=10&seed=0')
x2 = eng.prepare_inputs(imgs2[:512])
_, lg = eng.reference_loss(x2, torch.as_tensor(labels2[:512], device='cuda', dtype=torch.int32), training=True)
print('train-mode acc on train', (lg.argmax(1).cpu().numpy() == labels2[:512]).mean())

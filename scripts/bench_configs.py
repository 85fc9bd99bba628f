"""Measure the BASELINE.json configs that bench.py does not cover (one JSON line each):

  #1 SkDt single-trial random-search advisor on CPU: trials/hour through propose -> train ->
     evaluate -> dump_parameters on Fashion-MNIST-shaped synthetic data (60k train / 10k test, 28x28)
  #2 TfFeedForward-style MLP, 1 trial on 1 GPU: training images/s and trial wall time (same data)

  #3e VGG-small HPO trials end to end on 1 GPU: GP advisor -> VggSmall.train (10 epochs of 50k
     synthetic CIFAR-shaped images, batch 256, width 1.0) -> evaluate (10k) -> dump_parameters ->
     feedback, timed per trial (measured trials/hour; bench.py reports the steady-state step rate)

bench.py measures #1-#5 itself (#1, #2, #5 through rafiki_amd/utils/benchmarks.py); this script runs them
stand-alone.
"""
import argparse
import json
import os
import pickle
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TRAIN = 'synthetic://image?n={n}&size=28&channels=1&classes=10&seed=0'
TEST = 'synthetic://image?n={n}&size=28&channels=1&classes=10&seed=1'


def config1(n_train, n_test, trials):
    from rafiki_amd.utils.benchmarks import skdt_trials
    return skdt_trials(n_train, n_test, trials)


def config2(n_train, n_test, epochs):
    import torch
    from rafiki_amd.utils.benchmarks import mlp_trial
    dev = torch.device('cuda', 0) if torch.cuda.is_available() else torch.device('cpu')
    return mlp_trial(dev, n_train, n_test, epochs)


def config3(trials, epochs):
    import torch
    from rafiki_amd.advisor.advisor import make_advisor
    from rafiki_amd.constants import AdvisorType
    from rafiki_amd.model.model import load_model_class
    from rafiki_amd.models import model_file
    from rafiki_amd.parallel.context import TrialContext, use_context
    dev = torch.device('cuda', 0)
    clazz = load_model_class(open(model_file('VggSmall'), 'rb').read(), 'VggSmall')
    adv = make_advisor(clazz.get_knob_config(), AdvisorType.BTB_GP, seed=0)
    train = 'synthetic://image?n=50000&size=32&channels=3&classes=10&seed=0'
    test = 'synthetic://image?n=10000&size=32&channels=3&classes=10&seed=1'
    from rafiki_amd.model import dataset_utils
    dataset_utils.load_dataset_of_image_files(train, image_size=32)  # warm the generator cache
    dataset_utils.load_dataset_of_image_files(test, image_size=32)
    times, scores, phases = [], [], []
    with use_context(TrialContext(device=dev)):
        for _ in range(trials):
            t0 = time.perf_counter()
            knobs = adv.propose()
            knobs.update(epochs=epochs, batch_size=256, width_mult=1.0)
            m = clazz(**knobs)
            m.train(train)
            torch.cuda.synchronize()
            dtype = m._meta.get('dtype', 'fp32')
            t1 = time.perf_counter()
            s = m.evaluate(test)
            t2 = time.perf_counter()
            pickle.dumps(m.dump_parameters())
            t3 = time.perf_counter()
            m.destroy()
            adv.feedback(knobs, s)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
            phases.append({'train': round(t1 - t0, 3), 'evaluate': round(t2 - t1, 3), 'dump': round(t3 - t2, 3),
                           'rest': round(times[-1] - (t3 - t0), 3), 'train_detail': getattr(m, 'timings', {})})
            scores.append(s)
    steady = times[1:] or times
    per = sum(steady) / len(steady)
    return {'config': 'VGG-small 32x32x3 HPO trials end to end, GP advisor, 1 MI355X', 'metric': 'trials/hour',
            'value': round(3600.0 / per, 1), 'seconds_per_trial': round(per, 3),
            'first_trial_seconds': round(times[0], 3), 'trials': trials, 'phases_last_trial': phases[-1],
            'trial_definition': '{} epochs x 50000 images, batch 256, + eval 10000 + dump'.format(epochs),
            'best_score': max(scores), 'dtype': dtype,
            'data': 'synthetic CIFAR-shaped 50000+10000 32x32x3 (class-conditional), random-init weights'}


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--configs', default='1,2')
    ap.add_argument('--n_train', type=int, default=60000)
    ap.add_argument('--n_test', type=int, default=10000)
    ap.add_argument('--trials', type=int, default=3)
    ap.add_argument('--epochs', type=int, default=2)
    ap.add_argument('--vgg_trials', type=int, default=4)
    ap.add_argument('--vgg_epochs', type=int, default=10)
    a = ap.parse_args()
    if '3' in a.configs:
        print(json.dumps(config3(a.vgg_trials, a.vgg_epochs)), flush=True)
    if '1' in a.configs:
        print(json.dumps(config1(a.n_train, a.n_test, a.trials)), flush=True)
    if '2' in a.configs:
        print(json.dumps(config2(a.n_train, a.n_test, a.epochs)), flush=True)

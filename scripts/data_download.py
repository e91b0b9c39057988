# scripts/data_download.py -- fetch the pretraining corpus into the HF cache.
#
# Reference: Flink-ddd/pretraining-llm scripts/data_download.py:7-20
# (datasets.load_dataset(config.get('dataset_name', 'openwebtext'), split='train'),
# print example 0).  Same behaviour; without network access it explains how to
# proceed offline (local text via data_preprocess.py --text, or --synthetic).
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from config.config import default_config as config  # noqa: E402


def download_dataset():
    dataset_name = config.get('dataset_name', 'openwebtext')
    print(f"downloading / preparing dataset '{dataset_name}' ...")
    try:
        from datasets import load_dataset
        dataset = load_dataset(dataset_name, split='train')
    except Exception as e:  # no network in air-gapped clusters
        print(f"could not load '{dataset_name}': {type(e).__name__}: {e}")
        print("offline: use `python scripts/data_preprocess.py --text <files>` or `--synthetic N`")
        return None
    print("dataset cached. example:")
    print(dataset[0])
    return dataset


if __name__ == '__main__':
    download_dataset()

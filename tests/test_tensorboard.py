"""TensorBoard event files without tensorboard installed (reference engine.py:1057-1068)."""

import glob
import os

import torch

from common import run_distributed


def test_event_file_roundtrip(tmp_path):
    from deeperspeed_amd.utils.tb_writer import EventFileWriter, masked_crc32c, read_events
    from deeperspeed_amd.utils.tb_writer import _crc32c
    assert _crc32c(b"123456789") == 0xE3069283  # CRC-32C check value
    assert masked_crc32c(b"") == 0xA282EAD8
    w = EventFileWriter(str(tmp_path))
    for step in range(3):
        w.add_scalar("Train/Samples/train_loss", 1.5 - step, step)
    w.add_scalars("Train", {"lr": 0.1}, 7)
    w.close()
    ev = read_events(w.path)
    assert ev[:3] == [(0, "Train/Samples/train_loss", 1.5), (1, "Train/Samples/train_loss", 0.5),
                      (2, "Train/Samples/train_loss", -0.5)]
    assert ev[3][1] == "Train/lr" and abs(ev[3][2] - 0.1) < 1e-7 and ev[3][0] == 7


def _engine_tb(out_dir):
    import deeperspeed_amd as ds
    from simple_model import SimpleModel, random_batches
    model = SimpleModel(16)
    cfg = {"train_micro_batch_size_per_gpu": 4, "optimizer": {"type": "Adam", "params": {"lr": 1e-3}},
           "tensorboard": {"enabled": True, "output_path": out_dir, "job_name": "job"}}
    engine, _, _, _ = ds.initialize(model=model, model_parameters=model.parameters(), config_params=cfg)
    for x, y in random_batches(3, 4, 16):
        loss = engine(x, y)
        engine.backward(loss)
        engine.step()
    engine.summary_writer.flush()


def test_engine_writes_tensorboard(tmp_path):
    from deeperspeed_amd.utils.tb_writer import read_events
    run_distributed(_engine_tb, 1, str(tmp_path))
    files = glob.glob(os.path.join(tmp_path, "**", "events.out.tfevents.*"), recursive=True)
    assert files
    tags = {t for _, t, _ in read_events(files[0])}
    assert "Train/Samples/train_loss" in tags and "Train/Samples/lr" in tags

"""Restatement of pypanadapter_thread.py's `Data` ring (T:1400-1483) -- TEST INFRASTRUCTURE
ONLY (the reference class needs QtCore.QMutex and the NewtRap pacer, so it is restated here
without them).  `add` is T:1433-1457 minus the pacing sleep; `take` is the PSD worker's
get_data_start / data[:real_size] / get_data_end (T:1516-1520, 1459-1466)."""
import numpy as np


class Data:
    def __init__(self, chunk_size=8196 * 2, dtype=np.complex64):
        self.chunk_size = chunk_size
        self.max_size = self.chunk_size * 16              # T:1405
        self.data = np.zeros(self.max_size, dtype=dtype)  # new_complex, T:1420-1424
        self.size = 0
        self.real_size = 0
        self.total_size = 0

    def add(self, chunk):                                 # T:1433-1457
        length = len(chunk)
        new_size = self.size + length
        if new_size > self.max_size:
            self.size = 0
            new_size = length
        self.data[self.size:new_size] = chunk
        self.size = new_size
        self.real_size = max(self.real_size, self.size)
        self.total_size += length

    def take(self):                                       # T:1516-1520 with T:1462-1466
        size = self.real_size
        chunk = self.data[:size].copy()
        total = self.total_size
        self.size = 0
        self.real_size = 0
        self.total_size = 0
        return chunk, total

"""The admission benchmark behind bench.py (the driver's entry point).

* ``node``: rank 0's node under test (sysfs, accessible GPUs, advertised set)
  and its plugin instances;
* ``plugins``: the plugin under test (native daemon / Python oracle) behind a
  fake kubelet, and the GPU throughput check;
* ``admission``: one timed pod admission and the per-step records;
* ``extras``: the secondary measurements after the timed loop;
* ``coord``: rank coordination over gloo and the extras deadline;
* ``stats``: percentiles, tail attribution, allocation summaries.
"""

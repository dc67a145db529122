"""CPU oracle for the srpde-mi355x hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``superresolution_for_pdes_amd`` imports this
package; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may use it, and only as the checker / the timed CPU
baseline -- never as the product path.

* ``oracle.unet_ref``    -- functional torch-CPU restatement of the attention U-Net
                            (reference ``src/models.py:6-222``) and of one training
                            step (``src/train_enhanced.py:65-77``).
* ``oracle.poisson_ref`` -- numpy/scipy restatement of the 5-point Poisson assembly
                            and solve (``src/data_generation.py:35-159``,
                            ``src/enhanced_data_generation.py:47-191``) and of the
                            multi-level cascade (``src/resolution_comparison.py:13-229``).

Parity pinning: both restatements are checked against golden vectors produced by
importing the real reference in the build container (``tests/golden/make_golden.py``);
see ``tests/test_oracle_golden.py``.
"""

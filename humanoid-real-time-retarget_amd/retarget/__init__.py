"""Drop-in ``retarget`` package: solvers, geometry ops and robot tables of the
reference (retarget/), all arithmetic on the MI355X via librtg_hip."""

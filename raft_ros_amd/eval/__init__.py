from .validate import (validate_chairs, validate_sintel, validate_kitti, validate_synthetic,  # noqa: F401
                       create_sintel_submission, create_kitti_submission, run_validation)

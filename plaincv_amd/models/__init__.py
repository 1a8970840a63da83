"""Model families on the MI355X kernels (mirrors the reference's models/)."""

//! The few HIP runtime calls the safe layer needs to stage host states in HBM (libamdhip64).
use std::marker::PhantomData;
use std::os::raw::{c_int, c_void};
use std::ptr;

use super::GpuError;

const HIP_MEMCPY_HOST_TO_DEVICE: c_int = 1;
const HIP_MEMCPY_DEVICE_TO_HOST: c_int = 2;

#[link(name = "amdhip64")]
extern "C" {
    fn hipMalloc(ptr: *mut *mut c_void, size: usize) -> c_int;
    fn hipFree(ptr: *mut c_void) -> c_int;
    fn hipMemcpy(dst: *mut c_void, src: *const c_void, size: usize, kind: c_int) -> c_int;
    fn hipMemset(dst: *mut c_void, value: c_int, size: usize) -> c_int;
}

/// An owned device allocation of `len` values of a plain-old-data type (u8 / u32 / u64).
pub struct DeviceBuf<T: Copy + Default> {
    ptr: *mut c_void,
    len: usize,
    _t: PhantomData<T>,
}

fn hip(rc: c_int, what: &str) -> Result<(), GpuError> {
    if rc == 0 {
        Ok(())
    } else {
        Err(GpuError { code: rc, msg: format!("{} failed (hipError_t {})", what, rc) })
    }
}

impl<T: Copy + Default> DeviceBuf<T> {
    /// `hipMalloc` + `hipMemset(0)` of `len` values (at least one byte is allocated).
    pub fn zeroed(len: usize) -> Result<Self, GpuError> {
        let bytes = (len * std::mem::size_of::<T>()).max(8);
        let mut p = ptr::null_mut();
        hip(unsafe { hipMalloc(&mut p, bytes) }, "hipMalloc")?;
        let b = DeviceBuf { ptr: p, len, _t: PhantomData };
        hip(unsafe { hipMemset(p, 0, bytes) }, "hipMemset")?;
        Ok(b)
    }

    /// A device copy of `host`.
    pub fn from_host(host: &[T]) -> Result<Self, GpuError> {
        let b = Self::zeroed(host.len())?;
        if !host.is_empty() {
            let bytes = host.len() * std::mem::size_of::<T>();
            hip(unsafe { hipMemcpy(b.ptr, host.as_ptr() as *const c_void, bytes, HIP_MEMCPY_HOST_TO_DEVICE) },
                "hipMemcpy H2D")?;
        }
        Ok(b)
    }

    /// Copy back to the host (synchronous: waits for the work queued before it).
    pub fn to_host(&self) -> Result<Vec<T>, GpuError> {
        let mut v = vec![T::default(); self.len];
        if self.len > 0 {
            let bytes = self.len * std::mem::size_of::<T>();
            hip(unsafe { hipMemcpy(v.as_mut_ptr() as *mut c_void, self.ptr, bytes, HIP_MEMCPY_DEVICE_TO_HOST) },
                "hipMemcpy D2H")?;
        }
        Ok(v)
    }

    /// Device pointer (read-only use).
    pub fn as_ptr(&self) -> *const T {
        self.ptr as *const T
    }

    /// Device pointer (the library writes through it).
    pub fn as_mut_ptr(&self) -> *mut T {
        self.ptr as *mut T
    }
}

impl<T: Copy + Default> Drop for DeviceBuf<T> {
    fn drop(&mut self) {
        unsafe {
            hipFree(self.ptr);
        }
    }
}
